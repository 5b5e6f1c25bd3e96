// t-CSR temporal graph (TGL's ext_full.npz: indptr / indices / eid / ts, built by the absent
// tgb_gen_graph.py that utils.py:73 loads) and its "recent" neighbour sampler (TGL's C++ sampler_core,
// the build_ext of README.md:2, also absent from the reference), for gfx950.
//
// Build: every event contributes (src -> dst) and, with add_reverse, (dst -> src); one stable radix
// sort of (node << 36 | event id) keys (hipCUB) orders each node's row by event id, which is TGL's
// time order for a chronological stream (checked; reported through *chrono).
// Sample: one wave per root.  The row position of the cutoff (first entry with eid >= cut, or
// ts >= cut: TGL samples strictly before the root's time) is found by a 64-ary search — every lane
// probes one position per round, so a row of n entries takes ceil(log64 n) dependent rounds instead of
// log2 n — and the K entries before it are read by K lanes as one coalesced window, newest first.
// With cut = the batch's first event id the window is exactly LastNeighborLoader's ring row at the
// batch start (neighbor_loader.py:52-104: the K largest e_id per node), for any t.
#include <hipcub/hipcub.hpp>

#include "tgnx_common.h"

namespace tgnx {
namespace tcsr {

constexpr int EID_BITS = 36;

__global__ void build_keys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                           const float* __restrict__ t, int64_t E, int add_reverse, uint64_t* __restrict__ key,
                           uint32_t* __restrict__ val, int* __restrict__ flags) {
  const int64_t n = add_reverse ? 2 * E : E;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    const bool rev = j >= E;
    const int64_t e = rev ? j - E : j;
    const int64_t node = rev ? dst[e] : src[e];
    key[j] = ((uint64_t)node << EID_BITS) | (uint64_t)e;
    val[j] = (uint32_t)j;
    if (!rev && e > 0 && t[e] < t[e - 1]) flags[0] = 1;  // not chronological
  }
}

__global__ void build_fill(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                           const float* __restrict__ t, int64_t E, int64_t N, int64_t nnz,
                           const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                           int64_t* __restrict__ indptr, int64_t* __restrict__ indices, int64_t* __restrict__ eid,
                           float* __restrict__ ts) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= nnz; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t node = p < nnz ? (int64_t)(key[p] >> EID_BITS) : N;
    const int64_t prev = p > 0 ? (int64_t)(key[p - 1] >> EID_BITS) : -1;
    for (int64_t v = prev + 1; v <= node; ++v) indptr[v] = p;  // rows (prev, node] start at p
    if (p < nnz) {
      const int64_t j = val[p];
      const bool rev = j >= E;
      const int64_t e = rev ? j - E : j;
      indices[p] = rev ? src[e] : dst[e];
      eid[p] = e;
      ts[p] = t[e];
    }
  }
}

// first position b in [lo, hi) with key(b) >= cut (all before are < cut), wave-uniform
template <class KEY>
__device__ __forceinline__ int64_t wave_lower_bound(const KEY* __restrict__ k, int64_t lo, int64_t hi, KEY cut,
                                                    int lane) {
  while (hi - lo > 64) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t pos = lo + (int64_t)lane * step;
    const bool below = pos < hi && k[pos] < cut;
    const int cnt = __popcll(__ballot(below));
    // positions lo + i step, i < cnt, are below the cut: b lies in (lo + (cnt-1) step, lo + cnt step]
    if (cnt == 0) return lo;
    const int64_t nlo = lo + (int64_t)(cnt - 1) * step + 1;
    hi = min(hi, lo + (int64_t)cnt * step);
    lo = nlo;
  }
  const int64_t pos = lo + lane;
  const bool below = pos < hi && k[pos] < cut;
  return lo + __popcll(__ballot(below));
}

__global__ void __launch_bounds__(256) sample_recent(const int64_t* __restrict__ indptr,
                                                     const int64_t* __restrict__ indices,
                                                     const int64_t* __restrict__ eid, const float* __restrict__ ts,
                                                     int K, const int64_t* __restrict__ roots, int64_t Q, int mode,
                                                     const int64_t* __restrict__ cut_eid, int64_t cut_eid_all,
                                                     const float* __restrict__ cut_t, int64_t* __restrict__ out_nbr,
                                                     int64_t* __restrict__ out_eid, float* __restrict__ out_t,
                                                     int32_t* __restrict__ out_cnt) {
  const int lane = threadIdx.x & 63;
  for (int64_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < Q; q += (int64_t)gridDim.x * 4) {
    const int64_t v = roots[q];
    const int64_t lo = indptr[v], hi = indptr[v + 1];
    int64_t b;
    if (mode == 0) b = wave_lower_bound<int64_t>(eid, lo, hi, cut_eid ? cut_eid[q] : cut_eid_all, lane);
    else b = wave_lower_bound<float>(ts, lo, hi, cut_t[q], lane);
    const int64_t w0 = max(lo, b - (int64_t)K);
    const int c = (int)(b - w0);
    for (int j = lane; j < K; j += 64) {
      const bool ok = j < c;
      const int64_t p = ok ? b - 1 - j : lo;
      out_nbr[q * K + j] = ok ? indices[p] : -1;
      out_eid[q * K + j] = ok ? eid[p] : -1;
      out_t[q * K + j] = ok ? ts[p] : -1.0f;
    }
    if (lane == 0 && out_cnt) out_cnt[q] = c;
  }
}

// K <= 32: G-lane groups (G = 16 or 32), 64 / G roots per wave at once — the wave-per-root loop above left
// 64 - K lanes idle in the window read and walked its roots one after another, each root a chain of dependent
// loads (root -> indptr -> probes -> window).  A group's search is G-ary (ceil(log_G n) rounds: a wiki-shaped
// user row of <= 16 entries takes one, a hub page's thousands three); the groups of a wave diverge only in
// their round counts.  Consecutive groups take consecutive roots, so a wave's window stores are one
// contiguous run of (64 / G) K entries.
template <int G, class KEY>
__device__ __forceinline__ int64_t group_lower_bound(const KEY* __restrict__ k, int64_t lo, int64_t hi, KEY cut, int gl,
                                                     int gshift) {
  constexpr uint64_t GM = (1ull << G) - 1ull;
  while (hi - lo > G) {
    const int64_t step = (hi - lo + G - 1) / G;
    const int64_t pos = lo + (int64_t)gl * step;
    const bool below = pos < hi && k[pos] < cut;
    const int cnt = __popcll((__ballot(below) >> gshift) & GM);
    if (cnt == 0) return lo;
    const int64_t nlo = lo + (int64_t)(cnt - 1) * step + 1;
    hi = min(hi, lo + (int64_t)cnt * step);
    lo = nlo;
  }
  const int64_t pos = lo + gl;
  const bool below = pos < hi && k[pos] < cut;
  return lo + __popcll((__ballot(below) >> gshift) & GM);
}

template <int G>
__global__ void __launch_bounds__(256) sample_recent_g(const int64_t* __restrict__ indptr,
                                                       const int64_t* __restrict__ indices,
                                                       const int64_t* __restrict__ eid, const float* __restrict__ ts,
                                                       int K, const int64_t* __restrict__ roots, int64_t Q, int mode,
                                                       const int64_t* __restrict__ cut_eid, int64_t cut_eid_all,
                                                       const float* __restrict__ cut_t, int64_t* __restrict__ out_nbr,
                                                       int64_t* __restrict__ out_eid, float* __restrict__ out_t,
                                                       int32_t* __restrict__ out_cnt) {
  static_assert(G == 16 || G == 32, "group width");
  constexpr int GPW = 64 / G;
  const int lane = threadIdx.x & 63, gl = lane % G, grp = lane / G;
  const int64_t stride = (int64_t)gridDim.x * 4 * GPW;
  for (int64_t q = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * GPW + grp; q < Q; q += stride) {
    const int64_t v = roots[q];
    const int64_t ce = mode == 0 ? (cut_eid ? cut_eid[q] : cut_eid_all) : 0;
    const float ct = mode == 1 ? cut_t[q] : 0.f;
    const int64_t lo = indptr[v], hi = indptr[v + 1];
    const int64_t b = mode == 0 ? group_lower_bound<G, int64_t>(eid, lo, hi, ce, gl, grp * G)
                                : group_lower_bound<G, float>(ts, lo, hi, ct, gl, grp * G);
    const int c = (int)min((int64_t)K, b - lo);
    if (gl < K) {
      const bool ok = gl < c;
      const int64_t p = ok ? b - 1 - gl : lo;
      const int64_t o = q * K + gl;
      out_nbr[o] = ok ? indices[p] : -1;
      out_eid[o] = ok ? eid[p] : -1;
      out_t[o] = ok ? ts[p] : -1.0f;
    }
    if (gl == 0 && out_cnt) out_cnt[q] = c;
  }
}

struct BuildWs {
  size_t keys_in, keys_out, vals_in, vals_out, temp, flags, total, temp_bytes;
};
static BuildWs build_ws(int64_t nnz) {
  BuildWs w;
  size_t temp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)nnz, 0, 64);  // size query only
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  size_t o = 0;
  w.keys_in = o; o += al((size_t)nnz * 8);
  w.keys_out = o; o += al((size_t)nnz * 8);
  w.vals_in = o; o += al((size_t)nnz * 4);
  w.vals_out = o; o += al((size_t)nnz * 4);
  w.flags = o; o += 256;
  w.temp = o; o += al(temp);
  w.temp_bytes = temp;
  w.total = o;
  return w;
}

static int bits_for(int64_t n) {
  int b = 1;
  while (b < 62 && (int64_t(1) << b) <= n) ++b;
  return b;
}

}  // namespace tcsr
}  // namespace tgnx

using namespace tgnx;
using namespace tgnx::tcsr;

extern "C" {

size_t tgnx_tcsr_build_ws_bytes(int64_t num_events, int32_t add_reverse) {
  if (num_events <= 0) return 256;
  return build_ws(add_reverse ? 2 * num_events : num_events).total;
}

int tgnx_tcsr_build(const int64_t* src, const int64_t* dst, const float* t, int64_t num_events, int64_t num_nodes,
                    int32_t add_reverse, int64_t* indptr, int64_t* indices, int64_t* eid, float* ts, int32_t* chrono,
                    void* ws, size_t ws_bytes, void* stream) {
  TGNX_CHECK_ARG(num_events >= 0 && num_events < (int64_t(1) << EID_BITS) && num_nodes > 0 &&
                     num_nodes < (int64_t(1) << (63 - EID_BITS)),
                 "tgnx_tcsr_build: bad sizes");
  const int64_t nnz = add_reverse ? 2 * num_events : num_events;
  TGNX_CHECK_ARG(nnz < (int64_t(1) << 31), "tgnx_tcsr_build: more than 2^31 entries");
  TGNX_CHECK_ARG(indptr && ws && (num_events == 0 || (src && dst && t && indices && eid && ts)),
                 "tgnx_tcsr_build: null pointer");
  TGNX_CHECK_ARG(ws_bytes >= tgnx_tcsr_build_ws_bytes(num_events, add_reverse), "tgnx_tcsr_build: workspace too small");
  hipStream_t s = as_stream(stream);
  unsigned char* w = static_cast<unsigned char*>(ws);
  const BuildWs L = build_ws(nnz);
  uint64_t* kin = reinterpret_cast<uint64_t*>(w + L.keys_in);
  uint64_t* kout = reinterpret_cast<uint64_t*>(w + L.keys_out);
  uint32_t* vin = reinterpret_cast<uint32_t*>(w + L.vals_in);
  uint32_t* vout = reinterpret_cast<uint32_t*>(w + L.vals_out);
  int* flags = reinterpret_cast<int*>(w + L.flags);
  if (hipMemsetAsync(flags, 0, 256, s) != hipSuccess) {
    set_error("tgnx_tcsr_build: memset failed");
    return TGNX_EHIP;
  }
  const int grid = (int)std::min<int64_t>(4096, (std::max<int64_t>(nnz, 1) + 255) / 256);
  if (nnz > 0) {
    build_keys<<<grid, 256, 0, s>>>(src, dst, t, num_events, add_reverse, kin, vin, flags);
    TGNX_LAUNCH_CHECK("tcsr_build_keys");
    size_t temp = L.temp_bytes;
    const int end_bit = EID_BITS + bits_for(num_nodes);
    if (hipcub::DeviceRadixSort::SortPairs(w + L.temp, temp, kin, kout, vin, vout, (int)nnz, 0, end_bit, s) !=
        hipSuccess) {
      set_error("tgnx_tcsr_build: radix sort failed");
      return TGNX_EHIP;
    }
  }
  build_fill<<<grid, 256, 0, s>>>(src, dst, t, num_events, num_nodes, nnz, kout, vout, indptr, indices, eid, ts);
  TGNX_LAUNCH_CHECK("tcsr_build_fill");
  if (chrono) {  // offline preprocessing: a synchronous read of the flag is fine here
    int f = 0;
    if (hipMemcpyAsync(&f, flags, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_error("tgnx_tcsr_build: flag read failed");
      return TGNX_EHIP;
    }
    *chrono = f ? 0 : 1;
  }
  return TGNX_OK;
}

int tgnx_tcsr_sample(const int64_t* indptr, const int64_t* indices, const int64_t* eid, const float* ts,
                     int64_t num_nodes, int32_t K, const int64_t* roots, int64_t Q, int32_t mode, const int64_t* cut_eid,
                     int64_t cut_eid_all, const float* cut_t, int64_t* out_nbr, int64_t* out_eid, float* out_t,
                     int32_t* out_cnt, void* stream) {
  TGNX_CHECK_ARG(K > 0 && K <= 1024 && Q >= 0 && num_nodes > 0, "tgnx_tcsr_sample: bad sizes");
  TGNX_CHECK_ARG(mode == 0 || (mode == 1 && cut_t), "tgnx_tcsr_sample: mode 0 (eid < cut) or 1 (ts < cut_t[q])");
  if (Q == 0) return TGNX_OK;
  TGNX_CHECK_ARG(indptr && indices && eid && ts && roots && out_nbr && out_eid && out_t, "tgnx_tcsr_sample: null pointer");
  hipStream_t s = as_stream(stream);
  if (K <= 32) {
    const int G = K <= 16 ? 16 : 32, per = 4 * (64 / G);
    const int grid = (int)std::min<int64_t>(8192, (Q + per - 1) / per);
    if (G == 16)
      sample_recent_g<16><<<grid, 256, 0, s>>>(indptr, indices, eid, ts, K, roots, Q, mode, cut_eid, cut_eid_all, cut_t,
                                               out_nbr, out_eid, out_t, out_cnt);
    else
      sample_recent_g<32><<<grid, 256, 0, s>>>(indptr, indices, eid, ts, K, roots, Q, mode, cut_eid, cut_eid_all, cut_t,
                                               out_nbr, out_eid, out_t, out_cnt);
  } else {
    const int grid = (int)std::min<int64_t>(8192, (Q + 3) / 4);
    sample_recent<<<grid, 256, 0, s>>>(indptr, indices, eid, ts, K, roots, Q, mode, cut_eid, cut_eid_all, cut_t,
                                       out_nbr, out_eid, out_t, out_cnt);
  }
  TGNX_LAUNCH_CHECK("tcsr_sample_recent");
  return TGNX_OK;
}

}  // extern "C"
