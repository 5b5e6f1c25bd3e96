// Temporal neighbour ring on gfx950: LastNeighborLoader reset / sample / insert and the
// negative-destination sampler.  Reference: neighbor_loader.py:15-109, neg_sampler.py:3-23.
//
// Layout in HBM (identical to the reference's tensors so the drop-in class can expose
// them unchanged): nbr int64[N,K], eid int64[N,K], t fp32[N,K]; every row newest-first,
// empty slots eid = -1 at the tail.  All work here is index arithmetic on a few KB per
// call, so the kernels are shaped for latency (few launches, no host sync), not MFMA.
#include "tgnx_ring_dev.h"

namespace tgnx {


// ------------------------------------------------------------------ reset
__global__ void ring_reset_kernel(int64_t* __restrict__ eid, float* __restrict__ t, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    eid[i] = -1;
    t[i] = -1.0f;
  }
}

// ------------------------------------------------------------------ sample
// K1: one thread per query row: mark the query node and its valid neighbours in the node
// bitmap, count valid slots.
__global__ void ring_sample_mark(const int64_t* __restrict__ nbr, const int64_t* __restrict__ eid,
                                 const int64_t* __restrict__ n_id, int64_t q, int K,
                                 uint32_t* __restrict__ bm, int32_t* __restrict__ rowcnt) {
  int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= q) return;
  int64_t v = n_id[r];
  atomicOr(&bm[v >> 5], 1u << (v & 31));
  const int64_t* er = eid + v * K;
  const int64_t* nr = nbr + v * K;
  int c = 0;
  for (int j = 0; j < K; ++j) {
    if (er[j] >= 0) {
      int64_t u = nr[j];
      atomicOr(&bm[u >> 5], 1u << (u & 31));
      ++c;
    }
  }
  rowcnt[r] = c;
}

// K2: one workgroup: exclusive scan of the row counts (edge offsets) and an ordered walk
// of the bitmap that emits the sorted unique node list, writes assoc and re-zeroes the map.
__global__ void __launch_bounds__(1024) ring_sample_scan(int32_t* __restrict__ rowcnt, int64_t q,
                                                         uint32_t* __restrict__ bm, int64_t words,
                                                         int64_t* __restrict__ assoc, int64_t* __restrict__ out_nid,
                                                         int64_t cap_nodes, int64_t* __restrict__ counts) {
  __shared__ int sh[20];
  const int T = blockDim.x, tid = threadIdx.x;
  // rows
  int64_t rc = (q + T - 1) / T;
  int64_t r0 = tid * rc, r1 = min(q, r0 + rc);
  int s = 0;
  for (int64_t r = r0; r < r1; ++r) s += rowcnt[r];
  int tot_e;
  int base = block_excl_scan(s, sh, &tot_e);
  for (int64_t r = r0; r < r1; ++r) {
    int c = rowcnt[r];
    rowcnt[r] = base;
    base += c;
  }
  // bitmap
  int64_t wc = (words + T - 1) / T;
  int64_t w0 = tid * wc, w1 = min(words, w0 + wc);
  int pc = 0;
  for (int64_t w = w0; w < w1; ++w) pc += __popc(bm[w]);
  int tot_m;
  int rank = block_excl_scan(pc, sh, &tot_m);
  for (int64_t w = w0; w < w1; ++w) {
    uint32_t m = bm[w];
    if (!m) continue;
    bm[w] = 0u;
    while (m) {
      int b = __ffs(m) - 1;
      m &= m - 1;
      int64_t v = (w << 5) + b;
      if (rank < cap_nodes) out_nid[rank] = v;
      assoc[v] = rank;
      ++rank;
    }
  }
  if (tid == 0) {
    counts[0] = tot_m;
    counts[1] = tot_e;
  }
}

// K3: one thread per query row: write the compacted, relabelled edges.
__global__ void ring_sample_emit(const int64_t* __restrict__ nbr, const int64_t* __restrict__ eid,
                                 const float* __restrict__ tt, const int64_t* __restrict__ n_id, int64_t q, int K,
                                 const int32_t* __restrict__ rowoff, const int64_t* __restrict__ assoc,
                                 int64_t* __restrict__ out_ei, int64_t cap_e, int64_t* __restrict__ out_eid,
                                 float* __restrict__ out_t) {
  int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (r >= q) return;
  int64_t v = n_id[r];
  int64_t lv = assoc[v];
  int64_t o = rowoff[r];
  for (int j = 0; j < K; ++j) {
    int64_t e = eid[v * K + j];
    if (e < 0) continue;
    if (o < cap_e) {
      out_ei[o] = assoc[nbr[v * K + j]];
      out_ei[cap_e + o] = lv;
      out_eid[o] = e;
      out_t[o] = tt[v * K + j];
    }
    ++o;
  }
}

// ------------------------------------------------------------------ insert
__global__ void __launch_bounds__(1024) ring_insert_kernel(int64_t* __restrict__ nbr, int64_t* __restrict__ eid,
                                                           float* __restrict__ rt, int K,
                                                           const int64_t* __restrict__ src,
                                                           const int64_t* __restrict__ dst,
                                                           const float* __restrict__ ev_t, int B, int64_t cur,
                                                           int64_t* __restrict__ assoc) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int sh[20];
  ring_insert_block(nbr, eid, rt, K, src, dst, ev_t, B, cur, assoc, smem, sh);
}

// ------------------------------------------------------------------ negatives
__global__ void neg_sample_kernel(const int64_t* __restrict__ dst_nodes, int64_t n_dst,
                                  const int64_t* __restrict__ pos, int64_t B, uint64_t seed, uint64_t offset,
                                  int64_t* __restrict__ out) {
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= B) return;
  int64_t p = pos[i];
  int64_t v = dst_nodes[0];
  for (uint64_t attempt = 0; attempt < 64; ++attempt) {
    uint64_t h = hash4(seed, 0x6E656773ull, offset + (uint64_t)i, attempt);
    uint64_t r = (uint64_t)(((__uint128_t)(h >> 11) * (uint64_t)n_dst) >> 53);
    v = dst_nodes[r];
    if (v != p) break;
  }
  out[i] = v;
}

}  // namespace tgnx

using namespace tgnx;

extern "C" {

int tgnx_ring_reset(int64_t* eid, float* t, int64_t num_nodes, int32_t size, void* stream) {
  TGNX_CHECK_ARG(eid && t && num_nodes > 0 && size > 0, "tgnx_ring_reset: bad arguments");
  int64_t n = num_nodes * size;
  int64_t g64 = (n + 255) / 256;
  int grid = (int)(g64 < 4096 ? g64 : 4096);
  ring_reset_kernel<<<grid, 256, 0, as_stream(stream)>>>(eid, t, n);
  TGNX_LAUNCH_CHECK("ring_reset");
  return TGNX_OK;
}

size_t tgnx_ring_sample_ws_bytes(int64_t num_nodes, int64_t q) {
  size_t words = (size_t)((num_nodes + 31) / 32);
  size_t bm = ((words * 4 + 255) / 256) * 256;
  return bm + (size_t)(q + 1) * 4 + 256;
}

int tgnx_ring_sample(const int64_t* nbr, const int64_t* eid, const float* t, int64_t num_nodes, int32_t size,
                     const int64_t* n_id, int64_t q, int64_t* assoc, int64_t* out_nid, int64_t* out_ei,
                     int64_t* out_eid, float* out_t, int64_t cap_nodes, int64_t cap_edges, int64_t* counts,
                     void* ws, size_t ws_bytes, void* stream) {
  TGNX_CHECK_ARG(nbr && eid && t && assoc && counts && ws, "tgnx_ring_sample: null pointer");
  TGNX_CHECK_ARG(num_nodes > 0 && size > 0 && q >= 0, "tgnx_ring_sample: bad sizes");
  TGNX_CHECK_ARG(ws_bytes >= tgnx_ring_sample_ws_bytes(num_nodes, q), "tgnx_ring_sample: workspace too small");
  TGNX_CHECK_ARG(cap_nodes >= q * (1 + (int64_t)size) && cap_edges >= q * (int64_t)size,
                 "tgnx_ring_sample: output capacity below q*(1+K) / q*K");
  TGNX_CHECK_ARG(q < (1ll << 31) / (size + 1), "tgnx_ring_sample: query too large");
  hipStream_t s = as_stream(stream);
  int64_t words = (num_nodes + 31) / 32;
  uint32_t* bm = reinterpret_cast<uint32_t*>(ws);
  int32_t* rowcnt = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(ws) + ((words * 4 + 255) / 256) * 256);
  if (q > 0) {
    ring_sample_mark<<<(int)((q + 255) / 256), 256, 0, s>>>(nbr, eid, n_id, q, size, bm, rowcnt);
    TGNX_LAUNCH_CHECK("ring_sample_mark");
  }
  ring_sample_scan<<<1, 1024, 0, s>>>(rowcnt, q, bm, words, assoc, out_nid, cap_nodes, counts);
  TGNX_LAUNCH_CHECK("ring_sample_scan");
  if (q > 0) {
    ring_sample_emit<<<(int)((q + 255) / 256), 256, 0, s>>>(nbr, eid, t, n_id, q, size, rowcnt, assoc, out_ei,
                                                             cap_edges, out_eid, out_t);
    TGNX_LAUNCH_CHECK("ring_sample_emit");
  }
  return TGNX_OK;
}

int tgnx_ring_insert_max_batch(void) { return INSERT_MAX_B; }

int tgnx_ring_insert(int64_t* nbr, int64_t* eid, float* t, int64_t num_nodes, int32_t size, const int64_t* src,
                     const int64_t* dst, const float* ev_t, int64_t B, int64_t cur_e_id, int64_t* assoc,
                     void* stream) {
  TGNX_CHECK_ARG(nbr && eid && t && assoc, "tgnx_ring_insert: null pointer");
  TGNX_CHECK_ARG(size > 0 && size <= KMAX, "tgnx_ring_insert: ring size must be in [1, %d]", KMAX);
  if (B <= 0) return TGNX_OK;
  TGNX_CHECK_ARG(src && dst && ev_t, "tgnx_ring_insert: null event pointer");
  if (B > INSERT_MAX_B) {
    set_error("tgnx_ring_insert: batch %lld > %d", (long long)B, INSERT_MAX_B);
    return TGNX_ETOOBIG;
  }
  size_t shm = ring_insert_smem_bytes((int)B);
  ring_insert_kernel<<<1, 1024, shm, as_stream(stream)>>>(nbr, eid, t, size, src, dst, ev_t, (int)B, cur_e_id,
                                                         assoc);
  TGNX_LAUNCH_CHECK("ring_insert");
  return TGNX_OK;
}

int tgnx_neg_sample(const int64_t* dst_nodes, int64_t n_dst, const int64_t* pos, int64_t B, uint64_t seed,
                    uint64_t offset, int64_t* out, void* stream) {
  TGNX_CHECK_ARG(dst_nodes && pos && out && n_dst > 0 && B >= 0, "tgnx_neg_sample: bad arguments");
  if (B == 0) return TGNX_OK;
  neg_sample_kernel<<<(int)((B + 255) / 256), 256, 0, as_stream(stream)>>>(dst_nodes, n_dst, pos, B, seed, offset,
                                                                         out);
  TGNX_LAUNCH_CHECK("neg_sample");
  return TGNX_OK;
}

}  // extern "C"
