// Per-operator entry points ("msg_agg_last / mean, gru_update, predictor, edge_attn_fwd / bwd"):
// the TGN modules' operators one call each, for a torch caller that composes them itself (torch.ops.tgnx.*,
// csrc/tgnx_torch.cpp).  The fused train step (tgnx_tgn.hip) does not call these: it runs the same arithmetic
// inside its own launches.  Each section cites the reference module it restates.
//
//   tgnx_msg_agg          LastAggregator / MeanAggregator   modules/msg_agg.py:15-26
//   tgnx_memory_cell      TGNMemory.memory_updater          modules/memory_module.py:57,70-78,172 (GRUCell / RNNCell)
//   tgnx_link_predictor   LinkPredictor                     modules/decoder.py:12-27
//                         EdgePredictor (tile pairing)      model_utils.py:165-195
//   tgnx_edge_attn_fwd/bwd  TransformerConv's attention     modules/emb_module.py:21-29 (PyG TransformerConv)
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <math.h>

#include <algorithm>

#include "tgnx_common.h"

using namespace tgnx;

namespace {

constexpr int OPS_BLOCK = 256;
constexpr int WAVES = OPS_BLOCK / WAVE;
constexpr int HMAX = 8;  // attention heads per call

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
int key_bits(int64_t dim_size) {  // keys are in [0, dim_size] (dim_size = dropped)
  int b = 1;
  while (b < 62 && (int64_t(1) << b) <= dim_size) ++b;
  return b;
}

// ------------------------------------------------------------------ message aggregation (msg_agg.py:15-26)
// The messages are grouped by destination row with a stable radix sort of (index, position): row r's messages
// are then one contiguous run in ascending message order.  A wave per output row walks its run in that order:
//   last: the first message attaining the row's maximum t (torch_scatter scatter_max's argmax, CPU order), its
//         row copied; an empty row stays zero with argmax = n_msg (msg_agg.py:17-20);
//   mean: per column the sequential sum in message order (index_add's order) divided by the count, empty rows
//         zero (PyG scatter 'mean').
// Both are order-deterministic; an index outside [0, dim_size) is dropped and counted in *n_invalid.

struct AggWs {
  int64_t* keys_in;  // index, out-of-range entries keyed dim_size [n]
  int64_t* keys;     // sorted index [n]
  int64_t* pos;   // message positions in sorted order [n]
  int64_t* beg;   // run [beg, end) per row [dim_size]
  int64_t* end;
  void* sort_tmp;
  size_t sort_bytes;
};

size_t agg_sort_bytes(int64_t n, int64_t dim_size) {
  size_t bytes = 0;
  rocprim::counting_iterator<int64_t> pos0(0);
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const int64_t*)nullptr, (int64_t*)nullptr, pos0, (int64_t*)nullptr,
                            (size_t)n, 0, key_bits(dim_size));
  return bytes;
}

AggWs agg_ws(void* ws, int64_t n, int64_t dim_size) {
  char* p = reinterpret_cast<char*>(ws);
  AggWs w;
  w.keys_in = reinterpret_cast<int64_t*>(p);
  p += align256(n * 8);
  w.keys = reinterpret_cast<int64_t*>(p);
  p += align256(n * 8);
  w.pos = reinterpret_cast<int64_t*>(p);
  p += align256(n * 8);
  w.beg = reinterpret_cast<int64_t*>(p);
  p += align256(dim_size * 8);
  w.end = reinterpret_cast<int64_t*>(p);
  p += align256(dim_size * 8);
  w.sort_tmp = p;
  w.sort_bytes = agg_sort_bytes(n, dim_size);
  return w;
}

// out-of-range indices are keyed past every row (sorted to the end, never part of a run) and counted
__global__ void __launch_bounds__(OPS_BLOCK) agg_keys(const int64_t* index, int64_t n, int64_t dim_size,
                                                      int64_t* keys_in, int64_t* n_invalid) {
  const int64_t i = blockIdx.x * (int64_t)OPS_BLOCK + threadIdx.x;
  if (i >= n) return;
  const int64_t k = index[i];
  const bool ok = k >= 0 && k < dim_size;
  keys_in[i] = ok ? k : dim_size;
  if (!ok && n_invalid) atomicAdd(reinterpret_cast<unsigned long long*>(n_invalid), 1ull);
}

__global__ void __launch_bounds__(OPS_BLOCK) agg_runs(const int64_t* keys, int64_t n, int64_t dim_size,
                                                      int64_t* beg, int64_t* end) {
  const int64_t p = blockIdx.x * (int64_t)OPS_BLOCK + threadIdx.x;
  if (p >= n) return;
  const int64_t k = keys[p];
  if (k >= dim_size) return;
  if (p == 0 || keys[p - 1] != k) beg[k] = p;
  if (p == n - 1 || keys[p + 1] != k) end[k] = p + 1;
}

template <typename T>
__device__ __forceinline__ bool t_greater(T a, T b) { return a > b; }

// wave per output row
template <typename T>
__global__ void __launch_bounds__(OPS_BLOCK) agg_rows(int mode, const float* msg, int64_t n, int64_t dim,
                                                      const T* t, int64_t dim_size, const int64_t* pos,
                                                      const int64_t* beg, const int64_t* end, float* out,
                                                      int64_t* argmax) {
  const int64_t r = blockIdx.x * (int64_t)WAVES + (threadIdx.x >> 6);
  if (r >= dim_size) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = beg[r], e = end[r];
  float* o = out + r * dim;
  if (mode == 0) {
    // first maximum in message order: each lane the first max of its strided share, then the wave's
    // (t larger, or t equal and position smaller)
    int64_t best = -1;
    T bt{};
    for (int64_t p = b + lane; p < e; p += WAVE) {
      const int64_t m = pos[p];
      const T tv = t[m];
      if (best < 0 || t_greater(tv, bt)) {
        best = m;
        bt = tv;
      }
    }
    for (int o2 = 32; o2 > 0; o2 >>= 1) {
      const int64_t ob = __shfl_xor(best, o2, WAVE);
      const T ot = __shfl_xor(bt, o2, WAVE);
      if (ob >= 0 && (best < 0 || t_greater(ot, bt) || (!t_greater(bt, ot) && ob < best))) {
        best = ob;
        bt = ot;
      }
    }
    if (argmax && lane == 0) argmax[r] = best < 0 ? n : best;
    const float* src = best < 0 ? nullptr : msg + best * dim;
    for (int64_t c = lane; c < dim; c += WAVE) o[c] = src ? src[c] : 0.f;
    return;
  }
  const float cnt = (float)(e - b);
  for (int64_t c = lane; c < dim; c += WAVE) {
    float s = 0.f;
    for (int64_t p = b; p < e; ++p) s += msg[pos[p] * dim + c];
    o[c] = e > b ? __fdiv_rn(s, cnt) : 0.f;
  }
}

// ------------------------------------------------------------------ memory cell (memory_module.py:57,70-78,172)
// gi = x W_ih^T + b_ih, gh = h W_hh^T + b_hh on the MFMA GEMM (tgnx_gemm_f32), then the gates elementwise in
// torch's GRUCell form (r, z, n chunks): r = σ(gi_r + gh_r), z = σ(gi_z + gh_z), n = tanh(gi_n + r gh_n),
// h' = (h − n) z + n; the RNNCell (tanh): h' = tanh(gi + gh).
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void __launch_bounds__(OPS_BLOCK) cell_gates(int cell, int64_t M, int64_t D, const float* gi,
                                                        const float* gh, const float* h, float* h_out) {
  const int64_t x = blockIdx.x * (int64_t)OPS_BLOCK + threadIdx.x;
  if (x >= M * D) return;
  const int64_t m = x / D, d = x % D;
  if (cell == 1) {
    h_out[x] = tanhf(gi[x] + gh[x]);
    return;
  }
  const float* a = gi + m * 3 * D;
  const float* g = gh + m * 3 * D;
  const float rg = sigm(a[d] + g[d]);
  const float zg = sigm(a[D + d] + g[D + d]);
  const float ng = tanhf(a[2 * D + d] + rg * g[2 * D + d]);
  h_out[x] = (h[x] - ng) * zg + ng;
}

// ------------------------------------------------------------------ link predictor (decoder.py:12-27)
// hs = z_src W_src^T + b_src [n_src, D], hd = z_dst W_dst^T + b_dst [M, D] on the MFMA GEMM; then a wave per
// output row: out[i] = w_out · relu(hs[i mod n_src] + hd[i]) + b_out (σ for LinkPredictor; logits for
// EdgePredictor, whose negatives pair row i with source i mod B: model_utils.py:190 `tile`).
__global__ void __launch_bounds__(OPS_BLOCK) pred_rows(int64_t n_src, int64_t M, int64_t D, const float* hs,
                                                       const float* hd, const float* w_out, const float* b_out,
                                                       int sigmoid, float* out) {
  const int64_t i = blockIdx.x * (int64_t)WAVES + (threadIdx.x >> 6);
  if (i >= M) return;
  const int lane = threadIdx.x & 63;
  const float* a = hs + (i % n_src) * D;
  const float* b = hd + i * D;
  float s = 0.f;
  for (int64_t c = lane; c < D; c += WAVE) s += w_out[c] * fmaxf(a[c] + b[c], 0.f);
  s = wave_sum(s) + b_out[0];
  if (lane == 0) out[i] = sigmoid ? sigm(s) : s;
}

// ------------------------------------------------------------------ TransformerConv attention (PyG semantics)
// Destination i's incoming edges are rows [indptr[i], indptr[i+1]) of the per-edge k, v, e ([E, H*C]; q is per
// destination [n_dst, H*C]).  Per head h: a_p = q_i·(k_p + e_p) / sqrt(C); α = softmax over i's edges (max
// subtracted, + 1e-16 in the denominator, as torch_geometric.utils.softmax); out_i = Σ_p α_p (v_p + e_p).
// A wave per destination; lane owns channels x = lane + 64 r (r < NR), head x / C; per-head dot products are
// masked wave sums.  The scores are recomputed in each of the three passes (max, denominator, α and the
// weighted sum) rather than written and re-read.  Attention dropout is not applied (eval / dropout 0).
template <int NR>
struct AttnRow {
  float q[NR];
  int hd[NR];
  bool ok[NR];
};

template <int NR>
__device__ __forceinline__ void attn_scores(const AttnRow<NR>& row, const float* k, const float* e, int64_t p,
                                            int HC, int H, float sqrt_c, int lane, float* s) {
  float prod[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int x = lane + 64 * r;
    float kk = 0.f;
    if (row.ok[r]) {
      kk = k[p * HC + x];
      if (e) kk += e[p * HC + x];
    }
    prod[r] = row.q[r] * kk;
  }
#pragma unroll
  for (int h = 0; h < HMAX; ++h) {
    if (h >= H) break;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) v += (row.ok[r] && row.hd[r] == h) ? prod[r] : 0.f;
    s[h] = __fdiv_rn(wave_sum(v), sqrt_c);
  }
}

template <int NR>
__device__ __forceinline__ AttnRow<NR> attn_row(const float* q, int64_t i, int HC, int C, int lane) {
  AttnRow<NR> row;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int x = lane + 64 * r;
    row.ok[r] = x < HC;
    row.hd[r] = row.ok[r] ? x / C : 0;
    row.q[r] = row.ok[r] ? q[i * HC + x] : 0.f;
  }
  return row;
}

__device__ __forceinline__ void edge_range(const int64_t* indptr, int64_t i, int64_t E, int64_t& b, int64_t& e) {
  b = min(max(indptr[i], (int64_t)0), E);
  e = min(max(indptr[i + 1], b), E);
}

template <int NR>
__global__ void __launch_bounds__(OPS_BLOCK) attn_fwd(int64_t n_dst, int64_t E, int H, int C, const float* q,
                                                      const float* k, const float* v, const float* e,
                                                      const int64_t* indptr, float* out, float* alpha) {
  const int64_t i = blockIdx.x * (int64_t)WAVES + (threadIdx.x >> 6);
  if (i >= n_dst) return;
  const int lane = threadIdx.x & 63, HC = H * C;
  const float sqrt_c = (float)sqrt((double)C);
  const AttnRow<NR> row = attn_row<NR>(q, i, HC, C, lane);
  int64_t b, en;
  edge_range(indptr, i, E, b, en);
  float mx[HMAX], den[HMAX], s[HMAX];
#pragma unroll
  for (int h = 0; h < HMAX; ++h) {
    mx[h] = -INFINITY;
    den[h] = 0.f;
  }
  for (int64_t p = b; p < en; ++p) {
    attn_scores<NR>(row, k, e, p, HC, H, sqrt_c, lane, s);
#pragma unroll
    for (int h = 0; h < HMAX; ++h)
      if (h < H) mx[h] = fmaxf(mx[h], s[h]);
  }
  for (int64_t p = b; p < en; ++p) {
    attn_scores<NR>(row, k, e, p, HC, H, sqrt_c, lane, s);
#pragma unroll
    for (int h = 0; h < HMAX; ++h)
      if (h < H) den[h] += expf(s[h] - mx[h]);
  }
  float acc[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) acc[r] = 0.f;
  for (int64_t p = b; p < en; ++p) {
    attn_scores<NR>(row, k, e, p, HC, H, sqrt_c, lane, s);
    float a[HMAX];
#pragma unroll
    for (int h = 0; h < HMAX; ++h) a[h] = h < H ? __fdiv_rn(expf(s[h] - mx[h]), den[h] + 1e-16f) : 0.f;
    if (lane < H) {
      float al = a[0];
#pragma unroll
      for (int h = 1; h < HMAX; ++h)
        if (lane == h) al = a[h];
      alpha[p * H + lane] = al;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (!row.ok[r]) continue;
      const int x = lane + 64 * r;
      float vv = v[p * HC + x];
      if (e) vv += e[p * HC + x];
      float ah = a[0];
#pragma unroll
      for (int h = 1; h < HMAX; ++h)
        if (row.hd[r] == h) ah = a[h];
      acc[r] += vv * ah;
    }
  }
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (row.ok[r]) out[i * HC + lane + 64 * r] = acc[r];
}

// Backward of attn_fwd given dout [n_dst, H*C] and the forward's α [E, H]:
//   dα_p = dout_i · (v_p + e_p) per head;  ds_p = α_p (dα_p − Σ_p' α_p' dα_p');  g_p = ds_p / sqrt(C)
//   dq_i = Σ_p g_p (k_p + e_p);  dk_p = g_p q_i;  dv_p = α_p dout_i;  de_p = dk_p + dv_p
template <int NR>
__device__ __forceinline__ void attn_dalpha(const float* dout_r, const float* v, const float* e, int64_t p, int HC,
                                            int H, const AttnRow<NR>& row, int lane, float* da) {
  float prod[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int x = lane + 64 * r;
    float vv = 0.f;
    if (row.ok[r]) {
      vv = v[p * HC + x];
      if (e) vv += e[p * HC + x];
    }
    prod[r] = dout_r[r] * vv;
  }
#pragma unroll
  for (int h = 0; h < HMAX; ++h) {
    if (h >= H) break;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) s += (row.ok[r] && row.hd[r] == h) ? prod[r] : 0.f;
    da[h] = wave_sum(s);
  }
}

template <int NR>
__global__ void __launch_bounds__(OPS_BLOCK) attn_bwd(int64_t n_dst, int64_t E, int H, int C, const float* dout,
                                                      const float* q, const float* k, const float* v,
                                                      const float* e, const int64_t* indptr, const float* alpha,
                                                      float* dq, float* dk, float* dv, float* de) {
  const int64_t i = blockIdx.x * (int64_t)WAVES + (threadIdx.x >> 6);
  if (i >= n_dst) return;
  const int lane = threadIdx.x & 63, HC = H * C;
  const float sqrt_c = (float)sqrt((double)C);
  const AttnRow<NR> row = attn_row<NR>(q, i, HC, C, lane);
  float dout_r[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) dout_r[r] = row.ok[r] ? dout[i * HC + lane + 64 * r] : 0.f;
  int64_t b, en;
  edge_range(indptr, i, E, b, en);
  float S[HMAX], da[HMAX];
#pragma unroll
  for (int h = 0; h < HMAX; ++h) S[h] = 0.f;
  for (int64_t p = b; p < en; ++p) {
    attn_dalpha<NR>(dout_r, v, e, p, HC, H, row, lane, da);
#pragma unroll
    for (int h = 0; h < HMAX; ++h)
      if (h < H) S[h] += alpha[p * H + h] * da[h];
  }
  float dq_acc[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) dq_acc[r] = 0.f;
  for (int64_t p = b; p < en; ++p) {
    attn_dalpha<NR>(dout_r, v, e, p, HC, H, row, lane, da);
    float g[HMAX], al[HMAX];
#pragma unroll
    for (int h = 0; h < HMAX; ++h) {
      al[h] = h < H ? alpha[p * H + h] : 0.f;
      g[h] = h < H ? __fdiv_rn(al[h] * (da[h] - S[h]), sqrt_c) : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (!row.ok[r]) continue;
      const int x = lane + 64 * r;
      float gh = g[0], ah = al[0];
#pragma unroll
      for (int h = 1; h < HMAX; ++h)
        if (row.hd[r] == h) {
          gh = g[h];
          ah = al[h];
        }
      float kk = k[p * HC + x];
      if (e) kk += e[p * HC + x];
      dq_acc[r] += gh * kk;
      const float dkx = gh * row.q[r], dvx = ah * dout_r[r];
      dk[p * HC + x] = dkx;
      dv[p * HC + x] = dvx;
      if (de) de[p * HC + x] = dkx + dvx;
    }
  }
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (row.ok[r]) dq[i * HC + lane + 64 * r] = dq_acc[r];
}

template <template <int> class K, typename... A>
int attn_dispatch(int HC, int64_t n_dst, hipStream_t s, A... args) {
  const dim3 grid((unsigned)ceil_div(n_dst, WAVES));
  if (HC <= 64) hipLaunchKernelGGL(K<1>::fn, grid, dim3(OPS_BLOCK), 0, s, args...);
  else if (HC <= 128) hipLaunchKernelGGL(K<2>::fn, grid, dim3(OPS_BLOCK), 0, s, args...);
  else if (HC <= 256) hipLaunchKernelGGL(K<4>::fn, grid, dim3(OPS_BLOCK), 0, s, args...);
  else return TGNX_ETOOBIG;
  return TGNX_OK;
}
template <int NR>
struct FwdK {
  static constexpr auto fn = attn_fwd<NR>;
};
template <int NR>
struct BwdK {
  static constexpr auto fn = attn_bwd<NR>;
};

}  // namespace

extern "C" {

size_t tgnx_msg_agg_ws_bytes(int64_t n_msg, int64_t dim_size) {
  if (n_msg < 0 || dim_size < 0) return 0;
  return 3 * align256(n_msg * 8) + 2 * align256(dim_size * 8) + align256(agg_sort_bytes(n_msg, dim_size)) + 256;
}

int tgnx_msg_agg(int32_t mode, const float* msg, int64_t n_msg, int64_t dim, const int64_t* index, const void* t,
                 int32_t t_dtype, int64_t dim_size, float* out, int64_t* argmax, int64_t* n_invalid, void* ws,
                 size_t ws_bytes, void* stream) {
  TGNX_CHECK_ARG(mode == 0 || mode == 1, "tgnx_msg_agg: mode must be 0 (last) or 1 (mean)");
  TGNX_CHECK_ARG(n_msg >= 0 && dim >= 0 && dim_size >= 0 && n_msg < (int64_t(1) << 40) &&
                     dim_size < (int64_t(1) << 40),
                 "tgnx_msg_agg: bad sizes");
  TGNX_CHECK_ARG(mode == 1 || t_dtype == 0 || t_dtype == 1, "tgnx_msg_agg: t_dtype must be 0 (int64) or 1 (fp32)");
  if (dim_size == 0) return TGNX_OK;
  TGNX_CHECK_ARG(out && ws && (n_msg == 0 || (index && (dim == 0 || msg))) && (mode == 1 || n_msg == 0 || t),
                 "tgnx_msg_agg: null pointer");
  TGNX_CHECK_ARG(ws_bytes >= tgnx_msg_agg_ws_bytes(n_msg, dim_size), "tgnx_msg_agg: workspace too small");
  hipStream_t s = as_stream(stream);
  AggWs w = agg_ws(ws, n_msg, dim_size);
  TGNX_HIP_CHECK(hipMemsetAsync(w.beg, 0, dim_size * 8, s));
  TGNX_HIP_CHECK(hipMemsetAsync(w.end, 0, dim_size * 8, s));
  if (n_msg > 0) {
    const dim3 g((unsigned)ceil_div(n_msg, OPS_BLOCK));
    hipLaunchKernelGGL(agg_keys, g, dim3(OPS_BLOCK), 0, s, index, n_msg, dim_size, w.keys_in, n_invalid);
    TGNX_LAUNCH_CHECK("agg_keys");
    size_t bytes = w.sort_bytes;
    rocprim::counting_iterator<int64_t> pos0(0);
    TGNX_HIP_CHECK(rocprim::radix_sort_pairs(w.sort_tmp, bytes, (const int64_t*)w.keys_in, w.keys, pos0, w.pos,
                                             (size_t)n_msg, 0, key_bits(dim_size), s));
    hipLaunchKernelGGL(agg_runs, g, dim3(OPS_BLOCK), 0, s, (const int64_t*)w.keys, n_msg, dim_size, w.beg, w.end);
    TGNX_LAUNCH_CHECK("agg_runs");
  }
  const dim3 gr((unsigned)ceil_div(dim_size, WAVES));
  if (mode == 1 || t_dtype == 0)
    hipLaunchKernelGGL(agg_rows<int64_t>, gr, dim3(OPS_BLOCK), 0, s, (int)mode, msg, n_msg, dim,
                       reinterpret_cast<const int64_t*>(t), dim_size, (const int64_t*)w.pos, (const int64_t*)w.beg,
                       (const int64_t*)w.end, out, argmax);
  else
    hipLaunchKernelGGL(agg_rows<float>, gr, dim3(OPS_BLOCK), 0, s, (int)mode, msg, n_msg, dim,
                       reinterpret_cast<const float*>(t), dim_size, (const int64_t*)w.pos, (const int64_t*)w.beg,
                       (const int64_t*)w.end, out, argmax);
  TGNX_LAUNCH_CHECK("agg_rows");
  return TGNX_OK;
}

size_t tgnx_memory_cell_ws_bytes(int64_t M, int64_t d_in, int64_t D) {
  if (M <= 0 || d_in <= 0 || D <= 0) return 256;
  const size_t g = std::max(tgnx_gemm_f32_ws_bytes(M, 3 * D, d_in), tgnx_gemm_f32_ws_bytes(M, 3 * D, D));
  return 2 * align256(M * 3 * D * 4) + align256(g);
}

int tgnx_memory_cell(int32_t cell, int64_t M, int64_t d_in, int64_t D, const float* x, const float* h,
                     const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* h_out,
                     void* ws, size_t ws_bytes, void* stream) {
  TGNX_CHECK_ARG(cell == 0 || cell == 1, "tgnx_memory_cell: cell must be 0 (GRUCell) or 1 (RNNCell, tanh)");
  TGNX_CHECK_ARG(M >= 0 && d_in > 0 && D > 0 && M < (1 << 30) && d_in < (1 << 30) && D < (1 << 28),
                 "tgnx_memory_cell: bad sizes");
  if (M == 0) return TGNX_OK;
  TGNX_CHECK_ARG(x && h && w_ih && w_hh && h_out && ws, "tgnx_memory_cell: null pointer");
  TGNX_CHECK_ARG(ws_bytes >= tgnx_memory_cell_ws_bytes(M, d_in, D), "tgnx_memory_cell: workspace too small");
  const int64_t G = (cell == 0 ? 3 : 1) * D;
  char* p = reinterpret_cast<char*>(ws);
  float* gi = reinterpret_cast<float*>(p);
  float* gh = reinterpret_cast<float*>(p + align256(M * 3 * D * 4));
  void* gws = p + 2 * align256(M * 3 * D * 4);
  const size_t gbytes = ws_bytes - 2 * align256(M * 3 * D * 4);
  int rc = tgnx_gemm_f32(M, G, d_in, x, d_in, 0, w_ih, d_in, 1, gi, G, b_ih, 0, gws, gbytes, stream);
  if (rc != TGNX_OK) return rc;
  rc = tgnx_gemm_f32(M, G, D, h, D, 0, w_hh, D, 1, gh, G, b_hh, 0, gws, gbytes, stream);
  if (rc != TGNX_OK) return rc;
  hipLaunchKernelGGL(cell_gates, dim3((unsigned)ceil_div(M * D, OPS_BLOCK)), dim3(OPS_BLOCK), 0, as_stream(stream),
                     (int)cell, M, D, (const float*)gi, (const float*)gh, h, h_out);
  TGNX_LAUNCH_CHECK("cell_gates");
  return TGNX_OK;
}

size_t tgnx_link_predictor_ws_bytes(int64_t n_src, int64_t M, int64_t d_in, int64_t D) {
  if (n_src <= 0 || M <= 0 || d_in <= 0 || D <= 0) return 256;
  const size_t g = std::max(tgnx_gemm_f32_ws_bytes(n_src, D, d_in), tgnx_gemm_f32_ws_bytes(M, D, d_in));
  return align256(n_src * D * 4) + align256(M * D * 4) + align256(g);
}

int tgnx_link_predictor(int64_t n_src, int64_t M, int64_t d_in, int64_t D, const float* z_src, const float* z_dst,
                        const float* w_src, const float* b_src, const float* w_dst, const float* b_dst,
                        const float* w_out, const float* b_out, int32_t sigmoid, float* out, void* ws,
                        size_t ws_bytes, void* stream) {
  TGNX_CHECK_ARG(n_src >= 0 && M >= 0 && d_in > 0 && D > 0 && n_src < (1 << 30) && M < (1 << 30) &&
                     d_in < (1 << 30) && D < (1 << 30),
                 "tgnx_link_predictor: bad sizes");
  if (M == 0) return TGNX_OK;
  TGNX_CHECK_ARG(n_src > 0, "tgnx_link_predictor: rows to predict but no source rows");
  TGNX_CHECK_ARG(z_src && z_dst && w_src && w_dst && w_out && b_out && out && ws, "tgnx_link_predictor: null pointer");
  TGNX_CHECK_ARG(ws_bytes >= tgnx_link_predictor_ws_bytes(n_src, M, d_in, D), "tgnx_link_predictor: workspace too small");
  char* p = reinterpret_cast<char*>(ws);
  float* hs = reinterpret_cast<float*>(p);
  float* hd = reinterpret_cast<float*>(p + align256(n_src * D * 4));
  void* gws = p + align256(n_src * D * 4) + align256(M * D * 4);
  const size_t gbytes = ws_bytes - (align256(n_src * D * 4) + align256(M * D * 4));
  int rc = tgnx_gemm_f32(n_src, D, d_in, z_src, d_in, 0, w_src, d_in, 1, hs, D, b_src, 0, gws, gbytes, stream);
  if (rc != TGNX_OK) return rc;
  rc = tgnx_gemm_f32(M, D, d_in, z_dst, d_in, 0, w_dst, d_in, 1, hd, D, b_dst, 0, gws, gbytes, stream);
  if (rc != TGNX_OK) return rc;
  hipLaunchKernelGGL(pred_rows, dim3((unsigned)ceil_div(M, WAVES)), dim3(OPS_BLOCK), 0, as_stream(stream), n_src, M,
                     D, (const float*)hs, (const float*)hd, w_out, b_out, (int)sigmoid, out);
  TGNX_LAUNCH_CHECK("pred_rows");
  return TGNX_OK;
}

int tgnx_edge_attn_fwd(int64_t n_dst, int64_t n_edges, int32_t heads, int32_t channels, const float* q,
                       const float* k, const float* v, const float* e, const int64_t* indptr, float* out,
                       float* alpha, void* stream) {
  TGNX_CHECK_ARG(n_dst >= 0 && n_edges >= 0 && heads > 0 && heads <= HMAX && channels > 0,
                 "tgnx_edge_attn_fwd: bad sizes (1 <= heads <= %d)", HMAX);
  TGNX_CHECK_ARG((int64_t)heads * channels <= 256, "tgnx_edge_attn_fwd: heads * channels must be <= 256");
  if (n_dst == 0) return TGNX_OK;
  TGNX_CHECK_ARG(q && indptr && out && (n_edges == 0 || (k && v && alpha)), "tgnx_edge_attn_fwd: null pointer");
  const int rc = attn_dispatch<FwdK>(heads * channels, n_dst, as_stream(stream), n_dst, n_edges, (int)heads,
                                     (int)channels, q, k, v, e, indptr, out, alpha);
  if (rc != TGNX_OK) return rc;
  TGNX_LAUNCH_CHECK("attn_fwd");
  return TGNX_OK;
}

int tgnx_edge_attn_bwd(int64_t n_dst, int64_t n_edges, int32_t heads, int32_t channels, const float* dout,
                       const float* q, const float* k, const float* v, const float* e, const int64_t* indptr,
                       const float* alpha, float* dq, float* dk, float* dv, float* de, void* stream) {
  TGNX_CHECK_ARG(n_dst >= 0 && n_edges >= 0 && heads > 0 && heads <= HMAX && channels > 0,
                 "tgnx_edge_attn_bwd: bad sizes (1 <= heads <= %d)", HMAX);
  TGNX_CHECK_ARG((int64_t)heads * channels <= 256, "tgnx_edge_attn_bwd: heads * channels must be <= 256");
  if (n_dst == 0) return TGNX_OK;
  TGNX_CHECK_ARG(dout && q && indptr && dq && (n_edges == 0 || (k && v && alpha && dk && dv)) && (!e || de || !n_edges),
                 "tgnx_edge_attn_bwd: null pointer");
  const int rc = attn_dispatch<BwdK>(heads * channels, n_dst, as_stream(stream), n_dst, n_edges, (int)heads,
                                     (int)channels, dout, q, k, v, e, indptr, alpha, dq, dk, dv, de);
  if (rc != TGNX_OK) return rc;
  TGNX_LAUNCH_CHECK("attn_bwd");
  return TGNX_OK;
}

}  // extern "C"
