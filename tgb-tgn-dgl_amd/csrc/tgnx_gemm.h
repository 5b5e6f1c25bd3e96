// fp32 GEMM on v_mfma_f32_16x16x4_f32 for the small, latency-bound GEMMs of the TGN memory path
// (M ~ 10^2..10^4 rows, N, K ~ 10^2..10^3).  C[M,N] = Σ_k A(m,k) B(k,n), operands produced by loader
// functors (plain strided reads, or gathers that build the operand on the fly), the result handed to
// an epilogue functor per 64x64 tile.
//
// Workgroup = 256 threads (4 waves, each a 32x32 quadrant of 2x2 MFMA tiles), one 64x64 output tile
// and one K split.  Each workgroup loops over its k-chunks of KC <= 64: the next chunk's operands are
// loaded into registers while the current chunk's MFMAs run from LDS.
//   * direct GEMMs (S = 1): the workgroup runs the epilogue itself (fused gate math, biases, ...);
//   * deferred GEMMs (split-K): every split writes its partial tile, and a later launch
//     (gemm_fixup_kernel, one for all deferred GEMMs of a step) sums the partials in split order and
//     runs the epilogue.  No cross-workgroup synchronisation inside a launch: on gfx950 an
//     agent-scope release/acquire means an L2 writeback/invalidate per XCD, far costlier than the
//     kernel boundary that orders the partials here.
#pragma once
#include "tgnx_common.h"

namespace tgnx {

constexpr int GT = 64;        // output tile edge
constexpr int GKC = 64;       // k per chunk
constexpr int GPAD = GT + 1;  // LDS row pitch (floats)

typedef float f32x4_t __attribute__((ext_vector_type(4)));

struct GemmShape {
  int M, N, K, KC, S, tiles_m, tiles_n;  // capacities: the grid is sized from these
  int deferred;                          // 1: write partials for gemm_fixup_kernel
  const int *Mdev, *Ndev, *Kdev;         // optional runtime sizes on the device (<= capacities)
};
// direct GEMM: S = 1, the workgroup loops over all of K
inline GemmShape gemm_shape(int M, int N, int K, int KC, const int* Mdev = nullptr, const int* Ndev = nullptr,
                            const int* Kdev = nullptr) {
  GemmShape g;
  g.M = M; g.N = N; g.K = K;
  g.Mdev = Mdev; g.Ndev = Ndev; g.Kdev = Kdev;
  g.KC = KC > GKC ? GKC : KC;
  g.S = 1;
  g.deferred = 0;
  g.tiles_m = (M + GT - 1) / GT;
  g.tiles_n = (N + GT - 1) / GT;
  return g;
}
// deferred split-K GEMM: S <= smax splits, split s handles k-chunks s, s + S, ...
inline GemmShape gemm_shape_split(int M, int N, int K, int KC, const int* Mdev, const int* Ndev, const int* Kdev,
                                  int smax) {
  GemmShape g = gemm_shape(M, N, K, KC, Mdev, Ndev, Kdev);
  g.S = (K + g.KC - 1) / g.KC;
  if (g.S > smax) g.S = smax;
  if (g.S < 1) g.S = 1;
  g.deferred = 1;
  return g;
}
__host__ __device__ inline int gemm_blocks(const GemmShape& g) { return g.tiles_m * g.tiles_n * g.S; }
inline size_t gemm_partial_floats(const GemmShape& g) {
  return g.deferred ? (size_t)g.tiles_m * g.tiles_n * g.S * GT * GT : 0;
}

// Loader concept: `float operator()(int m_or_n, int k) const` (called only inside the runtime
// bounds), plus `static constexpr bool k_fast` (true when consecutive k are consecutive in memory)
// to pick the coalesced thread -> element mapping.  Epilogue concept:
// `void operator()(const float* Ct /*[GT][GPAD]*/, int m0, int n0, int M, int N) const`, run by all
// 256 threads of the workgroup, M / N the runtime bounds.

// Row-major operand: element (r, k) at p[r * ld + k]  (k_fast)
struct LoadRowK {
  const float* p;
  int rows, ks, ld;
  static constexpr bool k_fast = true;
  __device__ float operator()(int r, int k) const { return (r < rows && k < ks) ? p[(int64_t)r * ld + k] : 0.f; }
};
// Transposed operand: element (r, k) at p[k * ld + r]  (r fast)
struct LoadKRow {
  const float* p;
  int rows, ks, ld;
  static constexpr bool k_fast = false;
  __device__ float operator()(int r, int k) const { return (r < rows && k < ks) ? p[(int64_t)k * ld + r] : 0.f; }
};

constexpr int GEMM_SMEM_FLOATS = 2 * GKC * GPAD;
constexpr int GLD = GKC * GT / 256;  // operand elements per thread per chunk

struct GemmRt {
  int Mr, Nr, Kr, nchunk, Sr;
};
__device__ __forceinline__ GemmRt gemm_runtime(const GemmShape& g) {
  GemmRt r;
  r.Mr = g.Mdev ? min(*g.Mdev, g.M) : g.M;
  r.Nr = g.Ndev ? min(*g.Ndev, g.N) : g.N;
  r.Kr = g.Kdev ? min(*g.Kdev, g.K) : g.K;
  r.nchunk = (r.Kr + g.KC - 1) / g.KC;
  r.Sr = max(1, min(g.S, r.nchunk));
  return r;
}

// element mapping of a chunk load: thread tid, item i -> (row r, chunk column kk)
template <bool KFAST>
__device__ __forceinline__ void gemm_map(int tid, int i, int& r, int& kk) {
  const int x = tid + 256 * i;
  if (KFAST) { r = x / GKC; kk = x % GKC; } else { r = x % GT; kk = x / GT; }
}

// One workgroup of a GEMM (`bid` in [0, gemm_blocks(g))); `smem` holds GEMM_SMEM_FLOATS.
// A kernel may host several GEMMs by dispatching on block ranges.
template <class AL, class BL, class EPI>
__device__ __forceinline__ void gemm_body(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part,
                                          int bid, float* smem) {
  float (*As)[GPAD] = reinterpret_cast<float (*)[GPAD]>(smem);
  float (*Bs)[GPAD] = reinterpret_cast<float (*)[GPAD]>(smem + GKC * GPAD);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const GemmRt rt = gemm_runtime(g);
  const int tiles = g.tiles_m * g.tiles_n;
  const int tile = bid % tiles, s = bid / tiles;
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int m0 = tm * GT, n0 = tn * GT;
  if (m0 >= rt.Mr || n0 >= rt.Nr || s >= rt.Sr) return;  // the fixup skips such tiles / splits too
  const int wr = (wv >> 1) * 32, wc = (wv & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
  float ra[GLD], rb[GLD];
  auto fetch = [&](int ch) {  // chunk ch -> registers (every load in flight at once)
    const int k0 = ch * g.KC, kc = max(0, min(g.KC, rt.Kr - k0));
#pragma unroll
    for (int i = 0; i < GLD; ++i) {
      int r, kk;
      gemm_map<AL::k_fast>(tid, i, r, kk);
      ra[i] = (kk < kc && m0 + r < rt.Mr) ? al(m0 + r, k0 + kk) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < GLD; ++i) {
      int r, kk;
      gemm_map<BL::k_fast>(tid, i, r, kk);
      rb[i] = (kk < kc && n0 + r < rt.Nr) ? bl(n0 + r, k0 + kk) : 0.f;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < GLD; ++i) {
      int r, kk;
      gemm_map<AL::k_fast>(tid, i, r, kk);
      As[kk][r] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < GLD; ++i) {
      int r, kk;
      gemm_map<BL::k_fast>(tid, i, r, kk);
      Bs[kk][r] = rb[i];
    }
  };
  const int last = max(rt.nchunk, 1);
  fetch(s);
  stash();
  __syncthreads();
  for (int ch = s; ch < last; ch += g.S) {
    const int kc = max(0, min(g.KC, rt.Kr - ch * g.KC));
    const bool more = ch + g.S < last;
    if (more) fetch(ch + g.S);  // next chunk in flight during this chunk's MFMAs
    for (int kk = 0; kk < kc; kk += 4) {
      const float a0 = As[kk + lk][wr + li], a1 = As[kk + lk][wr + 16 + li];
      const float b0 = Bs[kk + lk][wc + li], b1 = Bs[kk + lk][wc + 16 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
    if (more) {
      stash();
      __syncthreads();
    }
  }
  if (g.deferred) {  // partial tile in register layout, summed by gemm_fixup_kernel
    f32x4_t* mine = reinterpret_cast<f32x4_t*>(part + ((size_t)tile * g.S + s) * GT * GT);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) mine[((wv * 2 + i) * 2 + j) * 64 + lane] = acc[i][j];
    return;
  }
  float (*Ct)[GPAD] = As;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ct[wr + 16 * i + lk * 4 + r][wc + 16 * j + li] = acc[i][j][r];
  __syncthreads();
  epi(&Ct[0][0], m0, n0, rt.Mr, rt.Nr);
}

template <class AL, class BL, class EPI>
__global__ void __launch_bounds__(256) gemm_kernel(GemmShape g, AL al, BL bl, EPI epi, float* part) {
  __shared__ __attribute__((aligned(16))) float smem[GEMM_SMEM_FLOATS];
  gemm_body(g, al, bl, epi, part, blockIdx.x, smem);
}

// Two independent GEMMs in one launch: blocks [0, gemm_blocks(g1)) run the first.
template <class AL1, class BL1, class EP1, class AL2, class BL2, class EP2>
__global__ void __launch_bounds__(256) gemm2_kernel(GemmShape g1, AL1 a1, BL1 b1, EP1 e1, float* p1, GemmShape g2,
                                                    AL2 a2, BL2 b2, EP2 e2, float* p2) {
  __shared__ __attribute__((aligned(16))) float smem[GEMM_SMEM_FLOATS];
  const int n1 = gemm_blocks(g1);
  if ((int)blockIdx.x < n1) gemm_body(g1, a1, b1, e1, p1, blockIdx.x, smem);
  else gemm_body(g2, a2, b2, e2, p2, blockIdx.x - n1, smem);
}

// ---------------------------------------------------------------- split-K fixup
template <class EPI>
struct GemmFix {
  GemmShape g;
  const float* part;
  EPI epi;
};
// one output tile of a deferred GEMM: Σ partials over the runtime splits in order, then the epilogue
template <class EPI>
__device__ void gemm_fix_tile(const GemmFix<EPI>& f, int tile, float* smem) {
  const GemmRt rt = gemm_runtime(f.g);
  const int tm = tile / f.g.tiles_n, tn = tile % f.g.tiles_n;
  const int m0 = tm * GT, n0 = tn * GT;
  if (m0 >= rt.Mr || n0 >= rt.Nr) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = (wv >> 1) * 32, wc = (wv & 1) * 32, li = lane & 15, lk = lane >> 4;
  float (*Ct)[GPAD] = reinterpret_cast<float (*)[GPAD]>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
      for (int q = 0; q < rt.Sr; ++q) {
        const f32x4_t* pq = reinterpret_cast<const f32x4_t*>(f.part + ((size_t)tile * f.g.S + q) * GT * GT);
        sum += pq[((wv * 2 + i) * 2 + j) * 64 + lane];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) Ct[wr + 16 * i + lk * 4 + r][wc + 16 * j + li] = sum[r];
    }
  __syncthreads();
  f.epi(&Ct[0][0], m0, n0, rt.Mr, rt.Nr);
}
template <class EPI>
__device__ __forceinline__ bool gemm_fix_dispatch(const GemmFix<EPI>& f, int& bid, float* smem) {
  const int nt = f.g.tiles_m * f.g.tiles_n;
  if (bid < nt) {
    gemm_fix_tile(f, bid, smem);
    return true;
  }
  bid -= nt;
  return false;
}
template <class EPI>
inline int gemm_fix_blocks(const GemmFix<EPI>& f) { return f.g.tiles_m * f.g.tiles_n; }

// Sum the partials of several deferred GEMMs (block ranges in argument order); blocks past them
// call `tail(bid)` (extra reductions that ride in the same launch).
template <class TAIL, class... E>
__global__ void __launch_bounds__(256) gemm_fixup_kernel(TAIL tail, GemmFix<E>... f) {
  __shared__ __attribute__((aligned(16))) float smem[GT * GPAD];
  int bid = blockIdx.x;
  if (!(gemm_fix_dispatch(f, bid, smem) || ...)) tail(bid);
}
struct NoTail {
  __device__ void operator()(int) const {}
};

// Epilogue: C[m, n] = v (+ bias[n]) (+= C if accumulate), row-major ldc.
struct EpiStore {
  float* C;
  const float* bias;
  int ldc, accumulate;
  __device__ void operator()(const float* Ct, int m0, int n0, int M, int N) const {
    for (int x = threadIdx.x; x < GT * GT; x += blockDim.x) {
      const int r = x / GT, cc = x % GT, m = m0 + r, n = n0 + cc;
      if (m < M && n < N) {
        float v = Ct[r * GPAD + cc] + (bias ? bias[n] : 0.f);
        float* o = C + (int64_t)m * ldc + n;
        *o = accumulate ? *o + v : v;
      }
    }
  }
};

template <class AL, class BL, class EPI>
static inline void gemm_launch(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part,
                               hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return;
  gemm_kernel<AL, BL, EPI><<<gemm_blocks(g), 256, 0, s>>>(g, al, bl, epi, part);
}
template <class AL1, class BL1, class EP1, class AL2, class BL2, class EP2>
static inline void gemm2_launch(const GemmShape& g1, const AL1& a1, const BL1& b1, const EP1& e1, float* p1,
                                const GemmShape& g2, const AL2& a2, const BL2& b2, const EP2& e2, float* p2,
                                hipStream_t s) {
  gemm2_kernel<AL1, BL1, EP1, AL2, BL2, EP2><<<gemm_blocks(g1) + gemm_blocks(g2), 256, 0, s>>>(g1, a1, b1, e1, p1, g2,
                                                                                              a2, b2, e2, p2);
}
template <class TAIL, class... E>
static inline void gemm_fixup_launch(int tail_blocks, const TAIL& tail, hipStream_t s, const GemmFix<E>&... f) {
  const int nb = (gemm_fix_blocks(f) + ... + 0) + tail_blocks;
  if (nb > 0) gemm_fixup_kernel<TAIL, E...><<<nb, 256, 0, s>>>(tail, f...);
}

}  // namespace tgnx
