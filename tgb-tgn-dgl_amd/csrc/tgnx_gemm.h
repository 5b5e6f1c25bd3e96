// Split-K fp32 GEMM on v_mfma_f32_16x16x4_f32 for the small, latency-bound GEMMs of the TGN memory
// path (M ~ 10^2..10^4 rows, N, K ~ 10^2).  C[M,N] = Σ_k A(m,k) B(k,n), operands produced by loader
// functors (plain strided reads, or gathers that build the operand on the fly), the result handed
// to an epilogue functor per 64x64 tile.
//
// Grid: tiles_m * tiles_n * S workgroups of 256 threads (4 waves, each a 32x32 quadrant of 2x2 MFMA
// tiles).  Workgroup (tile, s) owns k in [s*KC, (s+1)*KC): it loads its whole A/B chunk into LDS in
// one phase (every load in flight at once), runs KC/4 MFMA steps, and, when S > 1, writes its
// partial tile; the last of the S workgroups of a tile (atomic ticket) sums the S partials in
// order s = 0..S-1 (deterministic) into an LDS tile and runs the epilogue.  Tickets return to 0.
#pragma once
#include "tgnx_common.h"

namespace tgnx {

constexpr int GT = 64;        // output tile edge
constexpr int GKC = 64;       // max k per workgroup
constexpr int GPAD = GT + 1;  // LDS row pitch (floats)

typedef float f32x4_t __attribute__((ext_vector_type(4)));

struct GemmShape {
  int M, N, K, KC, S, tiles_m, tiles_n;  // capacities: the grid is sized from these
  const int *Mdev, *Ndev, *Kdev;         // optional runtime sizes on the device (<= capacities)
};
// S <= smax splits; split s handles k-chunks s, s + S, ... (so a large or device-sized K does not
// need a proportional grid).
inline GemmShape gemm_shape(int M, int N, int K, int KC, const int* Mdev = nullptr, const int* Ndev = nullptr,
                            const int* Kdev = nullptr, int smax = 16) {
  GemmShape g;
  g.M = M; g.N = N; g.K = K;
  g.Mdev = Mdev; g.Ndev = Ndev; g.Kdev = Kdev;
  g.KC = KC > GKC ? GKC : KC;
  g.S = (K + g.KC - 1) / g.KC;
  if (g.S > smax) g.S = smax;
  if (g.S < 1) g.S = 1;
  g.tiles_m = (M + GT - 1) / GT;
  g.tiles_n = (N + GT - 1) / GT;
  return g;
}
inline int gemm_blocks(const GemmShape& g) { return g.tiles_m * g.tiles_n * g.S; }
inline size_t gemm_partial_floats(const GemmShape& g) {
  return g.S > 1 ? (size_t)g.tiles_m * g.tiles_n * g.S * GT * GT : 0;
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

constexpr int GEMM_SMEM_FLOATS = 2 * GKC * GPAD + 1;

// One workgroup of a split-K GEMM (`bid` in [0, gemm_blocks(g))); `smem` holds GEMM_SMEM_FLOATS.
// A kernel may host several GEMMs by dispatching on block ranges (independent GEMMs of a step
// share a launch).
template <class AL, class BL, class EPI>
__device__ __forceinline__ void gemm_body(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part,
                                          int* ticket, int bid, float* smem) {
  float (*As)[GPAD] = reinterpret_cast<float (*)[GPAD]>(smem);
  float (*Bs)[GPAD] = reinterpret_cast<float (*)[GPAD]>(smem + GKC * GPAD);
  int& last = *reinterpret_cast<int*>(smem + 2 * GKC * GPAD);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int Mr = g.Mdev ? min(*g.Mdev, g.M) : g.M;
  const int Nr = g.Ndev ? min(*g.Ndev, g.N) : g.N;
  const int Kr = g.Kdev ? min(*g.Kdev, g.K) : g.K;
  const int nchunk = (Kr + g.KC - 1) / g.KC;
  const int Sr = max(1, min(g.S, nchunk));  // splits with work at run time
  const int tiles = g.tiles_m * g.tiles_n;
  const int tile = bid % tiles, s = bid / tiles;
  const int tm = tile / g.tiles_n, tn = tile % g.tiles_n;
  const int m0 = tm * GT, n0 = tn * GT;
  if (m0 >= Mr || n0 >= Nr || s >= Sr) return;  // all workgroups of such a tile / split leave together
  const int wr = (wv >> 1) * 32, wc = (wv & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = {0.f, 0.f, 0.f, 0.f};
  for (int ch = s; ch < max(nchunk, 1); ch += g.S) {
    const int k0 = ch * g.KC;
    const int kc = max(0, min(g.KC, Kr - k0));
    if (ch > s) __syncthreads();  // previous chunk's MFMA reads done
    // ---- one-phase operand load (A as As[k][m], B as Bs[k][n])
    for (int x = tid; x < GKC * GT; x += 256) {
      int r, kk;
      if (AL::k_fast) { r = x / GKC; kk = x % GKC; } else { r = x % GT; kk = x / GT; }
      As[kk][r] = (kk < kc && m0 + r < Mr) ? al(m0 + r, k0 + kk) : 0.f;
    }
    for (int x = tid; x < GKC * GT; x += 256) {
      int r, kk;
      if (BL::k_fast) { r = x / GKC; kk = x % GKC; } else { r = x % GT; kk = x / GT; }
      Bs[kk][r] = (kk < kc && n0 + r < Nr) ? bl(n0 + r, k0 + kk) : 0.f;
    }
    __syncthreads();
    // ---- MFMA: wave quadrant (wr, wc) of 32x32 = 2x2 tiles of 16x16
    for (int kk = 0; kk < kc; kk += 4) {
      const float a0 = As[kk + lk][wr + li], a1 = As[kk + lk][wr + 16 + li];
      const float b0 = Bs[kk + lk][wc + li], b1 = Bs[kk + lk][wc + 16 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  __syncthreads();  // As is reused as the output tile below
  float (*Ct)[GPAD] = As;
  if (Sr == 1) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) Ct[wr + 16 * i + lk * 4 + r][wc + 16 * j + li] = acc[i][j][r];
    __syncthreads();
    epi(&Ct[0][0], m0, n0, Mr, Nr);
    return;
  }
  // ---- split-K: partial in register layout, ticket, last arriver sums in order
  f32x4_t* mine = reinterpret_cast<f32x4_t*>(part + ((size_t)tile * g.S + s) * GT * GT);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) mine[((wv * 2 + i) * 2 + j) * 64 + lane] = acc[i][j];
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(&ticket[tile], 1) == Sr - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
      for (int q = 0; q < Sr; ++q) {
        const f32x4_t* pq = reinterpret_cast<const f32x4_t*>(part + ((size_t)tile * g.S + q) * GT * GT);
        sum += __builtin_nontemporal_load(&pq[((wv * 2 + i) * 2 + j) * 64 + lane]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) Ct[wr + 16 * i + lk * 4 + r][wc + 16 * j + li] = sum[r];
    }
  if (tid == 0) ticket[tile] = 0;
  __syncthreads();
  epi(&Ct[0][0], m0, n0, Mr, Nr);
}

template <class AL, class BL, class EPI>
__global__ void __launch_bounds__(256) gemm_splitk_kernel(GemmShape g, AL al, BL bl, EPI epi, float* part, int* ticket) {
  __shared__ __attribute__((aligned(16))) float smem[GEMM_SMEM_FLOATS];
  gemm_body(g, al, bl, epi, part, ticket, blockIdx.x, smem);
}

// Two independent GEMMs in one launch: blocks [0, gemm_blocks(g1)) run the first.
template <class AL1, class BL1, class EP1, class AL2, class BL2, class EP2>
__global__ void __launch_bounds__(256) gemm2_kernel(GemmShape g1, AL1 a1, BL1 b1, EP1 e1, float* p1, int* t1, GemmShape g2,
                                                    AL2 a2, BL2 b2, EP2 e2, float* p2, int* t2) {
  __shared__ __attribute__((aligned(16))) float smem[GEMM_SMEM_FLOATS];
  const int n1 = g1.tiles_m * g1.tiles_n * g1.S;
  if ((int)blockIdx.x < n1) gemm_body(g1, a1, b1, e1, p1, t1, blockIdx.x, smem);
  else gemm_body(g2, a2, b2, e2, p2, t2, blockIdx.x - n1, smem);
}

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
static inline void gemm_launch(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part, int* ticket,
                               hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return;
  gemm_splitk_kernel<AL, BL, EPI><<<gemm_blocks(g), 256, 0, s>>>(g, al, bl, epi, part, ticket);
}
template <class AL1, class BL1, class EP1, class AL2, class BL2, class EP2>
static inline void gemm2_launch(const GemmShape& g1, const AL1& a1, const BL1& b1, const EP1& e1, float* p1, int* t1,
                                const GemmShape& g2, const AL2& a2, const BL2& b2, const EP2& e2, float* p2, int* t2,
                                hipStream_t s) {
  gemm2_kernel<AL1, BL1, EP1, AL2, BL2, EP2><<<gemm_blocks(g1) + gemm_blocks(g2), 256, 0, s>>>(g1, a1, b1, e1, p1, t1,
                                                                                              g2, a2, b2, e2, p2, t2);
}

}  // namespace tgnx
