// fp32 GEMM on v_mfma_f32_16x16x4_f32 for the small, latency-bound GEMMs of the TGN memory path
// (M ~ 10^2..10^4 rows, N, K ~ 10^2..10^3).  C[M,N] = Σ_k A(m,k) B(k,n), operands produced by loader
// functors (plain strided reads, or gathers that build the operand on the fly), the result handed to
// an epilogue functor per output tile.
//
// Workgroup = 256 threads (4 waves in a 2x2 grid, each a (TM/2)x(TN/2) quadrant of 16x16 MFMA tiles),
// one TMxTN output tile and one K split; the tile config is a template parameter (GemmCfg).  At these
// sizes the step is latency-bound: a 64x64 tile leaves most of the 256 CUs idle and serialises the
// MFMAs of the whole K loop on a few CUs, so the TGN GEMMs use 32x32 tiles with 128-deep k-chunks
// (4x the workgroups, half the chunk round trips).  Each workgroup loops over its chunks: the next
// chunk's operands are loaded into registers while the current chunk's MFMAs run from LDS.
//   * direct GEMMs (S = 1): the workgroup runs the epilogue itself (fused gate math, biases, ...);
//   * deferred GEMMs (split-K): every split writes its partial tile, and a later launch
//     (gemm_fixup_kernel, one for all deferred GEMMs of a step) sums the partials in split order and
//     runs the epilogue.  No cross-workgroup synchronisation inside a launch: on gfx950 an
//     agent-scope release/acquire means an L2 writeback/invalidate per XCD, far costlier than the
//     kernel boundary that orders the partials here.
#pragma once
#include "tgnx_common.h"
#include <algorithm>
#include <type_traits>

namespace tgnx {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
// Write-through (sc1) stores for what a launch hands to the next one: a kernel boundary writes back the dirty
// L2 lines its predecessor left (MI355X_MICROARCH.md price list: + B / 6 TB/s), write-through stores leave none.
// (Vector stores: a relaxed agent-scope atomic store is global_store_dword sc1; 16 B: a buffer store, aux 16.)
__device__ __forceinline__ void st_wt(float* p, float v) {
  *p = v;
}
// 16 B at byte offset off (per lane) of the wave-uniform base, whose extent is bytes
__device__ __forceinline__ void st_wt4(float* base, int off, int bytes, f32x4_t v) {
  *reinterpret_cast<f32x4_t*>(reinterpret_cast<char*>(base) + off) = v;
}

template <int TM_, int TN_, int KC_, int PF_ = 1, bool WS_ = false, int DR_ = 0>
struct GemmCfg {
  static constexpr int TM = TM_, TN = TN_, KC = KC_;
  static constexpr int PF = PF_;  // k-chunks whose global loads are in flight ahead of the MFMAs
  // DR > 0 (with WS, 16x16 tiles): direct operands — each wave loads its k-slabs' MFMA operands straight into
  // registers, DR slabs (16 k each) per wave per round, every load of a round issued before the first MFMA;
  // no LDS staging, no barriers in the K loop (gemm_tile_direct)
  static constexpr int DR = DR_;
  // WS (wave split-K): every wave owns the whole TMxTN tile and every 4th 16-deep k-slab of a chunk;
  // the four partial tiles are summed through LDS in wave order.  Otherwise the 4 waves tile the output
  // 2x2, each a (TM/2)x(TN/2) quadrant over the whole chunk.
  static constexpr bool WS = WS_;
  static constexpr int FM = WS ? TM / 16 : TM / 32, FN = WS ? TN / 16 : TN / 32;  // 16x16 MFMA tiles per wave
  static constexpr int PK = KC + 4;                  // LDS row pitch of the k-contiguous operand rows
  static constexpr int PB = TN + 1;                  // LDS pitch of the C tile
  static constexpr int LA = TM * KC / 256, LB = TN * KC / 256;  // operand elements per thread per chunk
  static constexpr int SOP = (TM + TN) * PK, SRED = (WS ? 5 : 1) * TM * PB + 512;
  static constexpr int SMEM = SOP > SRED ? SOP : SRED;  // floats (operands; the C tile reuses them)
  static_assert(WS ? (TM % 16 == 0 && TN % 16 == 0 && KC % 64 == 0) : (TM % 32 == 0 && TN % 32 == 0 && KC % 16 == 0),
                "tile");
  static_assert(LA % 4 == 0 && LB % 4 == 0 && TM * TN % 256 == 0, "operand / C-tile split over 256 threads");
  static_assert(DR == 0 || (WS && TM == 16 && TN == 16), "direct operands: 16x16 wave-split tiles");
};
// The TGN step's GEMMs: 16x16 output tiles, wave split-K (GemmCfg::WS).  Each 16x16x4 fp32 MFMA issues
// for 32 cycles per SIMD, so a tile's time is set by its MFMA count on one CU: 32x32 tiles with the 2x2
// wave grid ran the GRU GEMM (M ~ 415, N = 400, K = 572) as 169 tiles of 4 x 143 chained MFMAs; 16x16 tiles
// spread the same MFMAs over 4x the workgroups (650 on 256 CUs) and the wave split cuts each wave's
// chain to K/64 slabs (tools/gemm_lab.hip: GRU 9.5 -> 8.2 us, dz0 7.9 -> 4.9 us per launch).
#ifndef TGNX_G32_T
#define TGNX_G32_T 16
#endif
#ifndef TGNX_G32_WS
#define TGNX_G32_WS 1
#endif
#ifndef TGNX_G32_KC
#define TGNX_G32_KC 64
#endif
#ifndef TGNX_G32_PF
#define TGNX_G32_PF 1
#endif
#ifndef TGNX_G32_DR
#define TGNX_G32_DR 2  // (same-box A/B, wiki step: staged 0.1030, 2 slabs per round 0.1024, 5 0.1037 ms)
#endif
using G32 = GemmCfg<TGNX_G32_T, TGNX_G32_T, TGNX_G32_KC, TGNX_G32_PF, TGNX_G32_WS, TGNX_G32_DR>;  // the TGN step's GEMMs
#ifndef TGNX_G32L_T
#define TGNX_G32L_T 16
#endif
#ifndef TGNX_G32L_WS
#define TGNX_G32L_WS 1
#endif
#ifndef TGNX_G32L_KC
#define TGNX_G32L_KC 64
#endif
#ifndef TGNX_G32L_PF
#define TGNX_G32L_PF 1
#endif
#ifndef TGNX_G32L_DR
#define TGNX_G32L_DR 3  // slabs per wave per load round (same-box A/B, wiki step: 9 (one round for K <= 576: 160 VGPRs, 3 waves per SIMD) 0.1073, 7 0.1060, 5 0.1045, 4 0.1045, 3 0.1041, staged path 0.1053 ms)
#endif
using G32L = GemmCfg<TGNX_G32L_T, TGNX_G32L_T, TGNX_G32L_KC, TGNX_G32L_PF, TGNX_G32L_WS, TGNX_G32L_DR>;  // long-K direct GEMMs (GRU, dz0, dX_enc)
// deferred split-K weight gradients (K = edges / nodes, split S ways): already S x tiles workgroups
#ifndef TGNX_GW_T
#define TGNX_GW_T 32
#endif
#ifndef TGNX_GW_WS
#define TGNX_GW_WS 0
#endif
#ifndef TGNX_GW_KC
#define TGNX_GW_KC 64
#endif
using GW = GemmCfg<TGNX_GW_T, TGNX_GW_T, TGNX_GW_KC, 1, TGNX_GW_WS>;
using G64 = GemmCfg<64, 64, 64>;   // large-M GEMMs (eval scoring)

#ifndef TGNX_GEMM_GRID_CAP
#define TGNX_GEMM_GRID_CAP 1024
#endif
struct GemmShape {
  int M, N, K, S, tiles_m, tiles_n;  // capacities: the grid is sized from these
  int tm, tn, kc;                    // the GemmCfg it was shaped for
  int deferred;                      // 1: write partials for gemm_fixup_kernel
  const int *Mdev, *Ndev, *Kdev;     // optional runtime sizes on the device (<= capacities)
  int cap;                           // grid cap (a multiple of 8; gemm_blocks)
};
// direct GEMM: S = 1, the workgroup loops over all of K
template <class CFG>
inline GemmShape gemm_shape(int M, int N, int K, const int* Mdev = nullptr, const int* Ndev = nullptr,
                            const int* Kdev = nullptr) {
  GemmShape g;
  g.M = M; g.N = N; g.K = K;
  g.Mdev = Mdev; g.Ndev = Ndev; g.Kdev = Kdev;
  g.tm = CFG::TM; g.tn = CFG::TN; g.kc = CFG::KC;
  g.S = 1;
  g.deferred = 0;
  g.tiles_m = (M + CFG::TM - 1) / CFG::TM;
  g.tiles_n = (N + CFG::TN - 1) / CFG::TN;
  g.cap = TGNX_GEMM_GRID_CAP;
  return g;
}
// the same GEMM with a smaller grid cap (its workgroups loop over the runtime tiles past it)
inline GemmShape with_cap(GemmShape g, int cap) {
  g.cap = (cap + 7) & ~7;
  return g;
}
// deferred split-K GEMM: S <= smax splits, split s handles k-chunks s, s + S, ...
template <class CFG>
inline GemmShape gemm_shape_split(int M, int N, int K, const int* Mdev, const int* Ndev, const int* Kdev, int smax) {
  GemmShape g = gemm_shape<CFG>(M, N, K, Mdev, Ndev, Kdev);
  g.S = (K + CFG::KC - 1) / CFG::KC;
  if (g.S > smax) g.S = smax;
  if (g.S < 1) g.S = 1;
  g.deferred = 1;
  return g;
}
// grid of a GEMM: tiles x splits of the CAPACITY shape, padded to a multiple of the 8 XCDs (see gemm_work),
// capped: capacities are worst cases (a 2-hop sample is sized for 2e5 rows and runs ~1e3), and
// dispatching 1e5 workgroups that exit at once cost ~80 us per launch; a workgroup loops over the
// runtime work in strides of the grid instead (gemm_body).
// (idle workgroups past the runtime tiles hold dispatch slots: 2048 -> 1024 shortened the step ~7 us on
// the wiki shape, stamps timeline; 512 lengthened the dW_gru launch, whose ~940 split blocks are all busy)
__host__ __device__ inline int gemm_blocks(const GemmShape& g) {
  const int full = (g.tiles_m * g.tiles_n * g.S + 7) & ~7;
  return full < g.cap ? full : g.cap;
}
inline size_t gemm_partial_floats(const GemmShape& g) {
  return g.deferred ? (size_t)g.tiles_m * g.tiles_n * g.S * g.tm * g.tn : 0;
}

// Loader concept: `static constexpr bool k_fast` (true when consecutive k are consecutive in memory,
// picks the coalesced thread -> element mapping) and either
//   * `float operator()(int m_or_n, int k) const` — a load whose address needs no other load, or
//   * a two-phase gather: `using Idx`, `static constexpr bool row_idx`, `Idx index(int r, int k)`
//     (the index loads: node ids, event ids, ...) and `float load(const Idx&, int r, int k)`.
// The body issues every index load of a chunk before any data load (row_idx: once per tile, before
// the K loop).  A data load whose address depends on an index load in the same batch would force
// `s_waitcnt vmcnt(0)` per element — vmcnt retires in issue order — and serialise the chunk.
// Loaders are called with in-range (clamped) r and k; out-of-range elements are zeroed afterwards.
//
// Epilogue concept: `template <class T> void operator()(const T& t) const` with T a GemmTile<TM, TN>,
// run by all 256 threads of the workgroup; t(r, cc) is C[m0 + r][n0 + cc] for r < tm, cc < tn, M / N
// the runtime bounds.  The tile shape is compile-time so epilogues can issue every gather of the
// tile before their first store (the compiler cannot hoist loads over stores that may alias).
template <int TM_, int TN_>
struct GemmTile {
  static constexpr int tm = TM_, tn = TN_, pitch = TN_ + 1, per = TM_ * TN_ / 256;  // elements per thread
  const float* c;
  int m0, n0, M, N;
  float* scratch;  // >= 512 floats of LDS past the tile, free for the epilogue
  __device__ float operator()(int r, int cc) const { return c[r * pitch + cc]; }
  __device__ int tile_row() const { return m0 / tm; }
  // element i of this thread: tile row / column
  __device__ static int row_of(int i) { return (threadIdx.x + 256 * i) / tn; }
  __device__ static int col_of(int i) { return (threadIdx.x + 256 * i) % tn; }
};

// Loaded values are never selected against at load time (`c ? v : 0.f` lets the compiler sink the
// load into a branch whose join waits on it): the body zeroes out-of-range elements when it stashes
// them, and loaders express constant entries arithmetically (v * 0/1 + c).
__device__ __forceinline__ float f01(bool b) { return b ? 1.0f : 0.0f; }
// lane l's value of a per-lane index (any lane l of the wave)
__device__ __forceinline__ int shfl_idx(int v, int l) { return __shfl(v, l, 64); }
__device__ __forceinline__ int64_t shfl_idx(int64_t v, int l) {
  return (int64_t)(((uint64_t)(uint32_t)__shfl((int)(v >> 32), l, 64) << 32) | (uint64_t)(uint32_t)__shfl((int)v, l, 64));
}
template <class T>
__device__ __forceinline__ T shfl_idx(const T& v, int) { return v; }  // (index types without a lane value)

template <class L, class = void>
struct LoaderTraits {  // plain loader
  using Idx = int;
  static constexpr bool row_idx = true;
  __device__ static Idx index(const L&, int, int) { return 0; }
  __device__ static float load(const L& l, const Idx&, int r, int k) { return l(r, k); }
  __device__ static float4 load4(const L& l, const Idx&, int r, int k) { return l.load4(r, k); }
};
template <class L>
struct LoaderTraits<L, std::void_t<typename L::Idx>> {  // two-phase gather
  using Idx = typename L::Idx;
  static constexpr bool row_idx = L::row_idx;
  __device__ static Idx index(const L& l, int r, int k) { return l.index(r, k); }
  __device__ static float load(const L& l, const Idx& i, int r, int k) { return l.load(i, r, k); }
  __device__ static float4 load4(const L& l, const Idx& i, int r, int k) { return l.load4(i, r, k); }
};
// 16-B operand loads.  A k_fast loader may also provide `bool vec4() const` (runtime: every k segment
// of its rows starts at a multiple of 4 floats and every row is 16-B aligned) and `load4` (elements k..k+3
// of row r, k % 4 == 0, one global_load_dwordx4).  When vec4() holds for both operands and K % 4 == 0,
// the body fetches such operands 4 k per lane (a quarter of the load instructions; ~1 us per launch on
// the TGN GEMMs, tools/gemm_lab.hip) and stashes them with one ds_write_b128.
template <class L, class = void>
struct HasVec4 : std::false_type {};
template <class L>
struct HasVec4<L, std::void_t<decltype(std::declval<const L&>().vec4())>> : std::integral_constant<bool, L::k_fast> {};
template <class L>
__device__ __forceinline__ bool vec_ok(const L& l) {
  if constexpr (HasVec4<L>::value) return l.vec4();
  else return true;
}
__device__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Row-major operand: element (r, k) at p[r * ld + k]  (k_fast).  rows x ks bound the buffer (the body
// clamps r, k to the GEMM's runtime bounds, which every call site keeps within it).
struct LoadRowK {
  const float* p;
  int rows, ks, ld;
  static constexpr bool k_fast = true;
  __device__ float operator()(int r, int k) const { return p[(int64_t)min(r, rows - 1) * ld + min(k, ks - 1)]; }
  __device__ bool vec4() const { return (ld & 3) == 0 && (ks & 3) == 0 && al16(p); }
  __device__ float4 load4(int r, int k) const {
    return *reinterpret_cast<const float4*>(p + (int64_t)min(r, rows - 1) * ld + min(k, ks - 4));
  }
};
// Transposed operand: element (r, k) at p[k * ld + r]  (r fast)
struct LoadKRow {
  const float* p;
  int rows, ks, ld;
  static constexpr bool k_fast = false;
  __device__ float operator()(int r, int k) const { return p[(int64_t)min(k, ks - 1) * ld + min(r, rows - 1)]; }
};

struct GemmRt {
  int Mr, Nr, Kr, nchunk, Sr;
};
template <class CFG>
__device__ __forceinline__ GemmRt gemm_runtime(const GemmShape& g) {
  GemmRt r;
  r.Mr = g.Mdev ? min(*g.Mdev, g.M) : g.M;
  r.Nr = g.Ndev ? min(*g.Ndev, g.N) : g.N;
  r.Kr = g.Kdev ? min(*g.Kdev, g.K) : g.K;
  r.nchunk = (r.Kr + CFG::KC - 1) / CFG::KC;
  r.Sr = max(1, min(g.S, r.nchunk));
  return r;
}

// element mapping of a chunk load: thread tid, item i -> (row r, chunk column kk).  k-fast operands:
// consecutive threads take consecutive k (coalesced loads, conflict-free b32 LDS stores); r-fast
// operands: consecutive threads take consecutive rows and each thread 4 consecutive k (coalesced
// loads per k, one b128 LDS store).
template <bool KFAST, int ROWS, int KC>
__device__ __forceinline__ void gemm_map(int tid, int i, int& r, int& kk) {
  if (KFAST) {
    const int x = tid + 256 * i;
    r = x / KC; kk = x % KC;
  } else {
    const int x = tid + 256 * (i >> 2);
    r = x % ROWS; kk = 4 * (x / ROWS) + (i & 3);
  }
}

// XCD-aware work mapping.  Workgroups are dispatched round-robin over the 8 XCDs (bid % 8) and each
// XCD has its own L2, so with a plain bid -> tile order every XCD fetches all of A and all of B from
// the fabric (PMC: 16.7 MB per launch for the GRU GEMM against ~4 MB algorithmic).  Here XCD x takes
// the contiguous run [x T/8, (x+1) T/8) of a grouped tile order (GROUP m-tiles per column sweep), so
// it touches ~T/8 tiles packed in a GROUP x (T/8/GROUP) rectangle.  Splits are the slowest index.
// The order is laid over the RUNTIME tile counts (capacities are worst-case: 6,600 rows against
// ~415 at run time would put every live tile on one XCD); partial-buffer offsets stay in capacity
// tile numbering.
#ifndef TGNX_GEMM_GROUP
#define TGNX_GEMM_GROUP 4
#endif
constexpr int GEMM_GROUP = TGNX_GEMM_GROUP;
struct GemmWork {
  int tile, s, tm, tn;
  bool ok;
};
template <int TM, int TN>
__device__ __forceinline__ GemmWork gemm_work(const GemmShape& g, int Mr, int Nr, int Sr, int bid) {
  GemmWork w;
  const int tmr = (Mr + TM - 1) / TM, tnr = (Nr + TN - 1) / TN;
  const int tiles = tmr * tnr, T = tiles * Sr, per = (T + 7) >> 3;
  const int L = (bid & 7) * per + (bid >> 3);
  w.ok = (bid >> 3) < per && L < T && tiles > 0;
  const int s = w.ok ? L / tiles : 0, tl = w.ok ? L - s * tiles : 0;
  // GEMM_GROUP 0: groups of half the m-tiles, so that each XCD's ~T/8 tiles form a (tmr/2) x (tnr/4) rectangle
  // (A fetched by 4 XCDs, B by 2, instead of a 4-row strip across ~all of B)
  const int GG = GEMM_GROUP > 0 ? GEMM_GROUP : max(1, (tmr + 1) >> 1);
  const int gw = GG * max(tnr, 1), grp = tl / gw, m_first = grp * GG;
  const int gsz = max(1, min(tmr - m_first, GG)), r = tl - grp * gw;
  w.s = s;
  w.tm = m_first + r % gsz;
  w.tn = r / gsz;
  w.tile = w.tm * g.tiles_n + w.tn;
  return w;
}

// Direct-operand 16x16 tile (CFG::DR > 0, wave split-K): wave w owns k-slabs w, w + 4, ... (16 k each), and
// lane (li, lk) of an MFMA step q takes k = 16 slab + 4 lk + q — the same slabs, k order, accumulator chains
// and wave-order combine as the LDS-staged WS path, so the results are bit-identical to it.  Each lane loads
// its 4 consecutive k of row m0 + li (A) and column n0 + li (B) per slab straight into registers: a float4
// for 16-B operands (V), else 4 scalars; DR slabs per round, all of a round's loads issued before its first
// MFMA (k past K: both entries selected to zero at use).  The chunked loop waited a whole load latency per
// 64-deep chunk (stash, barrier, MFMAs, barrier): the GRU GEMM's K = 572 paid 9 of them per tile.
// Epilogue prefetch (direct tiles): an epilogue with `struct Pre` and
//   `template <class RI> Pre pre(int m0, int n0, int M, int N, RI rowidx) const`
// gets its loads issued with the tile's first operand round (rowidx(r): the A loader's index of tile row r,
// e.g. the node of a gathered row) and is then called as epi(tile, pre): its gathers ride in the operand
// rounds instead of adding their own dependent rounds after the MFMAs.
template <class E, class = void>
struct HasPre : std::false_type {};
template <class E>
struct HasPre<E, std::void_t<typename E::Pre>> : std::true_type {};
struct NoPre {};
template <class E, class = void>
struct PreOf {
  using type = NoPre;
};
template <class E>
struct PreOf<E, std::void_t<typename E::Pre>> {
  using type = typename E::Pre;
};

template <class CFG, bool V, class AL, class BL, class EPI>
__device__ __forceinline__ void gemm_tile_direct(const GemmShape& g, const GemmRt& rt, const AL& al, const BL& bl,
                                                 const EPI& epi, float* part, int bid, float* smem) {
  constexpr int TM = 16, TN = 16, PB = CFG::PB, DR = CFG::DR;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const GemmWork wk = gemm_work<TM, TN>(g, rt.Mr, rt.Nr, rt.Sr, bid);
  const int tile = wk.tile, s = wk.s;
  const int m0 = wk.tm * TM, n0 = wk.tn * TN;
  if (!wk.ok || m0 >= rt.Mr || n0 >= rt.Nr || s >= rt.Sr) return;
  const int li = lane & 15, lk = lane >> 4;
  using TA = LoaderTraits<AL>;
  using TB = LoaderTraits<BL>;
  static_assert(TA::row_idx && TB::row_idx, "direct operands: row-indexed loaders");
  constexpr bool AV = V && HasVec4<AL>::value, BV = V && HasVec4<BL>::value;
  const int ra = min(m0 + li, rt.Mr - 1), rb = min(n0 + li, rt.Nr - 1);
  const typename TA::Idx ia = TA::index(al, ra, 0);
  const typename TB::Idx ib = TB::index(bl, rb, 0);
  const int klast = max(rt.Kr - 1, 0), k4last = max(rt.Kr - 4, 0);
  const int nslab = (rt.Kr + 15) >> 4;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  float a[DR][4], b[DR][4];
  auto issue = [&](int j0) {  // one round: DR slabs of this wave, every load issued
#pragma unroll
    for (int u = 0; u < DR; ++u) {
      const int k = 16 * (j0 + 4 * rt.Sr * u) + 4 * lk;
      if constexpr (AV) {
        const float4 v = TA::load4(al, ia, ra, min(k, k4last));
        a[u][0] = v.x; a[u][1] = v.y; a[u][2] = v.z; a[u][3] = v.w;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[u][q] = TA::load(al, ia, ra, min(k + q, klast));
      }
      if constexpr (BV) {
        const float4 v = TB::load4(bl, ib, rb, min(k, k4last));
        b[u][0] = v.x; b[u][1] = v.y; b[u][2] = v.z; b[u][3] = v.w;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) b[u][q] = TB::load(bl, ib, rb, min(k + q, klast));
      }
    }
  };
  // the epilogue's gathers with the first round (they need only the row indices the operands wait for too)
  using PreT = typename PreOf<EPI>::type;
  PreT pre{};
  if constexpr (HasPre<EPI>::value) pre = epi.pre(m0, n0, rt.Mr, rt.Nr, [&](int r) { return shfl_idx(ia, r); });
  // split s of S takes the 64-deep chunks s, s + S, ...: this wave's slabs 4 s + wv, 4 (s + S) + wv, ...
  const int SS = 4 * rt.Sr;
  for (int j0 = 4 * s + wv; j0 < nslab; j0 += SS * DR) {  // rounds of DR slabs of this wave
    issue(j0);
#pragma unroll
    for (int u = 0; u < DR; ++u) {
      const int j = j0 + SS * u;
      if (j < nslab) {  // (wave-uniform)
        const int k = 16 * j + 4 * lk;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool kin = k + q < rt.Kr;  // (the staged path's zero padding, on both operands)
          const float aq = kin ? a[u][q] : 0.f, bq = kin ? b[u][q] : 0.f;
          if (q & 1) acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(aq, bq, acc2, 0, 0, 0);
          else acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aq, bq, acc, 0, 0, 0);
        }
      }
    }
  }
  // wave partials -> LDS, summed in wave order (as the WS path)
  float* red = smem;  // [4][TM][PB], then Ct [TM][PB]
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wv * TM * PB + (lk * 4 + r) * PB + li] = acc[r] + acc2[r];
  __syncthreads();
  float* Ct = red + 4 * TM * PB;
  {
    const int x = tid, o = (x / TN) * PB + x % TN;  // TM * TN == 256: one element per thread
    const float v = ((red[o] + red[TM * PB + o]) + red[2 * TM * PB + o]) + red[3 * TM * PB + o];
    if (g.deferred) st_wt(part + ((size_t)tile * g.S + s) * TM * TN + x, v);
    else Ct[o] = v;
  }
  if (g.deferred) return;
  __syncthreads();
  if constexpr (HasPre<EPI>::value) epi(GemmTile<TM, TN>{Ct, m0, n0, rt.Mr, rt.Nr, Ct + TM * PB}, pre);
  else epi(GemmTile<TM, TN>{Ct, m0, n0, rt.Mr, rt.Nr, Ct + TM * PB});
}

// One work item (virtual block `bid` of the XCD-grouped order) of a GEMM; `smem` holds CFG::SMEM floats.
template <class CFG, bool V, class AL, class BL, class EPI>
__device__ __forceinline__ void gemm_tile(const GemmShape& g, const GemmRt& rt, const AL& al, const BL& bl,
                                          const EPI& epi, float* part, int bid, float* smem) {
  if constexpr (CFG::DR > 0 && V) {  // (element-wise operands: the staged path — measured faster there, the
                                      // comment-shaped 2-hop GRU at Qm = 302: 26 vs 41 us per launch)
    gemm_tile_direct<CFG, V>(g, rt, al, bl, epi, part, bid, smem);
    return;
  }
  constexpr int TM = CFG::TM, TN = CFG::TN, KC = CFG::KC, FM = CFG::FM, FN = CFG::FN;
  constexpr int PK = CFG::PK, PB = CFG::PB, LA = CFG::LA, LB = CFG::LB;
  float* As = smem;            // [TM][PK]: row m, k contiguous
  float* Bs = smem + TM * PK;  // [TN][PK]: row n, k contiguous
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const GemmWork wk = gemm_work<TM, TN>(g, rt.Mr, rt.Nr, rt.Sr, bid);
  const int tile = wk.tile, s = wk.s;
  const int m0 = wk.tm * TM, n0 = wk.tn * TN;
  if (!wk.ok || m0 >= rt.Mr || n0 >= rt.Nr || s >= rt.Sr) return;  // the fixup skips such tiles / splits too
  const int wr = CFG::WS ? 0 : (wv >> 1) * (TM / 2), wc = CFG::WS ? 0 : (wv & 1) * (TN / 2);
  const int li = lane & 15, lk = lane >> 4;
  f32x4_t acc[FM][FN], acc2[FM][FN];  // acc2: second accumulator chain of the WS path (odd MFMA steps)
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = acc2[i][j] = {0.f, 0.f, 0.f, 0.f};
  constexpr int PF = CFG::PF;
  float ra[PF][LA], rb[PF][LB];
  // chunk ch -> register slot p (every load of the slot in flight at once)
  using TA = LoaderTraits<AL>;
  using TB = LoaderTraits<BL>;
  typename TA::Idx ia[LA];
  typename TB::Idx ib[LB];
  const int mlast = rt.Mr - 1, nlast = rt.Nr - 1, klast = max(rt.Kr - 1, 0), k4last = max(rt.Kr - 4, 0);
  // 16-B operands (V: vec_ok for both and K % 4 == 0): item i of the thread = float4 (row x / (KC/4),
  // k 4 (x % (KC/4))), x = tid + 256 i
  constexpr bool AV = V && HasVec4<AL>::value, BV = V && HasVec4<BL>::value;
  static_assert(!AV || TA::row_idx, "16-B loads need a row index");
  static_assert(!BV || TB::row_idx, "16-B loads need a row index");
  // index phase (every index load of the operand issued before any data load)
  auto index_a = [&](int k0) {
    if constexpr (AV) {
#pragma unroll
      for (int i = 0; i < LA / 4; ++i) ia[i] = TA::index(al, min(m0 + (tid + 256 * i) / (KC / 4), mlast), 0);
    } else {
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        int r, kk;
        gemm_map<AL::k_fast, TM, KC>(tid, i, r, kk);
        ia[i] = TA::index(al, min(m0 + r, mlast), min(k0 + kk, klast));
      }
    }
  };
  auto index_b = [&](int k0) {
    if constexpr (BV) {
#pragma unroll
      for (int i = 0; i < LB / 4; ++i) ib[i] = TB::index(bl, min(n0 + (tid + 256 * i) / (KC / 4), nlast), 0);
    } else {
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        int r, kk;
        gemm_map<BL::k_fast, TN, KC>(tid, i, r, kk);
        ib[i] = TB::index(bl, min(n0 + r, nlast), min(k0 + kk, klast));
      }
    }
  };
  if (TA::row_idx) index_a(0);
  if (TB::row_idx) index_b(0);
  // chunk ch -> registers: clamped in-range loads (out-of-range elements are zeroed in stash)
  auto fetch = [&](float* fa, float* fb, int ch) {
    const int k0 = ch * KC;
    if (!TA::row_idx) index_a(k0);
    if (!TB::row_idx) index_b(k0);
    if constexpr (AV) {
#pragma unroll
      for (int i = 0; i < LA / 4; ++i) {
        const int x = tid + 256 * i;
        const float4 v = TA::load4(al, ia[i], min(m0 + x / (KC / 4), mlast), min(k0 + 4 * (x % (KC / 4)), k4last));
        fa[4 * i] = v.x; fa[4 * i + 1] = v.y; fa[4 * i + 2] = v.z; fa[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < LA; ++i) {
        int r, kk;
        gemm_map<AL::k_fast, TM, KC>(tid, i, r, kk);
        fa[i] = TA::load(al, ia[i], min(m0 + r, mlast), min(k0 + kk, klast));
      }
    }
    if constexpr (BV) {
#pragma unroll
      for (int i = 0; i < LB / 4; ++i) {
        const int x = tid + 256 * i;
        const float4 v = TB::load4(bl, ib[i], min(n0 + x / (KC / 4), nlast), min(k0 + 4 * (x % (KC / 4)), k4last));
        fb[4 * i] = v.x; fb[4 * i + 1] = v.y; fb[4 * i + 2] = v.z; fb[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < LB; ++i) {
        int r, kk;
        gemm_map<BL::k_fast, TN, KC>(tid, i, r, kk);
        fb[i] = TB::load(bl, ib[i], min(n0 + r, nlast), min(k0 + kk, klast));
      }
    }
  };
  // registers -> LDS, zeroing elements outside the runtime bounds (rlast: last valid row of the tile
  // origin r0; kc: valid k of the chunk)
  auto stash1 = [&](float* S, const float* rv, auto mode, auto rows, auto cnt, int r0, int rlast, int kc) {
    constexpr int ROWS = decltype(rows)::value, CNT = decltype(cnt)::value, MODE = decltype(mode)::value;
    if constexpr (MODE == 2) {  // 16-B items
#pragma unroll
      for (int i = 0; i < CNT / 4; ++i) {
        const int x = tid + 256 * i, r = x / (KC / 4), kk = 4 * (x % (KC / 4));
        const bool rok = r0 + r <= rlast;
        *reinterpret_cast<f32x4_t*>(S + r * PK + kk) =
            f32x4_t{(rok && kk < kc) ? rv[4 * i] : 0.f, (rok && kk + 1 < kc) ? rv[4 * i + 1] : 0.f,
                    (rok && kk + 2 < kc) ? rv[4 * i + 2] : 0.f, (rok && kk + 3 < kc) ? rv[4 * i + 3] : 0.f};
      }
    } else if constexpr (MODE == 1) {  // k-fast scalars
#pragma unroll
      for (int i = 0; i < CNT; ++i) {
        int r, kk;
        gemm_map<true, ROWS, KC>(tid, i, r, kk);
        S[r * PK + kk] = (kk < kc && r0 + r <= rlast) ? rv[i] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < CNT; i += 4) {
        int r, kk;
        gemm_map<false, ROWS, KC>(tid, i, r, kk);
        const bool rok = r0 + r <= rlast;
        *reinterpret_cast<f32x4_t*>(S + r * PK + kk) =
            f32x4_t{(rok && kk < kc) ? rv[i] : 0.f, (rok && kk + 1 < kc) ? rv[i + 1] : 0.f,
                    (rok && kk + 2 < kc) ? rv[i + 2] : 0.f, (rok && kk + 3 < kc) ? rv[i + 3] : 0.f};
      }
    }
  };
  auto stash = [&](const float* fa, const float* fb, int ch) {
    const int kc = max(0, min(KC, rt.Kr - ch * KC));
    stash1(As, fa, std::integral_constant<int, AV ? 2 : AL::k_fast ? 1 : 0>{}, std::integral_constant<int, TM>{},
           std::integral_constant<int, LA>{}, m0, mlast, kc);
    stash1(Bs, fb, std::integral_constant<int, BV ? 2 : BL::k_fast ? 1 : 0>{}, std::integral_constant<int, TN>{},
           std::integral_constant<int, LB>{}, n0, nlast, kc);
  };
  // k permutation inside a 16-deep slab: MFMA step q of lane (li, lk) takes k = 4 lk + q, so each
  // lane's operands for 4 steps are one b128 LDS read (same permutation for A and B)
  auto slab = [&](int kk, f32x4_t* a, f32x4_t* b) {
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const f32x4_t*>(As + (wr + 16 * i + li) * PK + kk + 4 * lk);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const f32x4_t*>(Bs + (wc + 16 * j + li) * PK + kk + 4 * lk);
  };
  auto mfma_chunk = [&]() {
    if constexpr (CFG::WS) {  // this wave's slabs wv, wv + 4, ... of the chunk
#pragma unroll
      for (int u = 0; u < KC / 64; ++u) {
        f32x4_t a[FM], b[FN];
        slab(16 * (wv + 4 * u), a, b);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) {
              if (q & 1) acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc2[i][j], 0, 0, 0);
              else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
            }
      }
      return;
    }
    f32x4_t a[2][FM], b[2][FN];
    slab(0, a[0], b[0]);
#pragma unroll
    for (int it = 0; it < KC / 16; ++it) {
      const int cur = it & 1;
      if (it + 1 < KC / 16) slab(16 * (it + 1), a[cur ^ 1], b[cur ^ 1]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur][i][q], b[cur][j][q], acc[i][j], 0, 0, 0);
    }
  };
  // PF-deep pipeline: the loads of the next PF chunks of this split are in flight while a chunk
  // is stashed and multiplied (PF = 4 at KC = 128: every load of a K <= 512 GEMM issued up front)
  const int last = max(rt.nchunk, 1);
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (s + p * g.S < last) fetch(ra[p], rb[p], s + p * g.S);
  for (int c0 = s; c0 < last; c0 += PF * g.S) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int ch = c0 + p * g.S;
      if (ch < last) {
        stash(ra[p], rb[p], ch);
        __syncthreads();
        if (ch + PF * g.S < last) fetch(ra[p], rb[p], ch + PF * g.S);
        mfma_chunk();
        __syncthreads();
      }
    }
  }
  if constexpr (CFG::WS) {  // wave partials -> LDS, summed in wave order into the C tile
    float* red = smem;  // [4][TM][PB], then Ct [TM][PB]
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          red[wv * TM * PB + (16 * i + lk * 4 + r) * PB + 16 * j + li] = acc[i][j][r] + acc2[i][j][r];
    __syncthreads();
    float* Ct = red + 4 * TM * PB;
    constexpr int PER = TM * TN / 256;
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int x = tid + 256 * e, o = (x / TN) * PB + x % TN;
      const float v = ((red[o] + red[TM * PB + o]) + red[2 * TM * PB + o]) + red[3 * TM * PB + o];
      if (g.deferred) st_wt(part + ((size_t)tile * g.S + s) * TM * TN + x, v);  // row-major partial tile
      else Ct[o] = v;
    }
    if (g.deferred) return;
    __syncthreads();
    epi(GemmTile<TM, TN>{Ct, m0, n0, rt.Mr, rt.Nr, Ct + TM * PB});
    return;
  }
  if (g.deferred) {  // partial tile in register layout, summed by gemm_fixup_kernel
    float* mine = part + ((size_t)tile * g.S + s) * TM * TN;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) st_wt4(mine, (((wv * FM + i) * FN + j) * 64 + lane) * 16, TM * TN * 4, acc[i][j]);
    return;
  }
  float* Ct = smem;  // [TM][PB]
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ct[(wr + 16 * i + lk * 4 + r) * PB + wc + 16 * j + li] = acc[i][j][r];
  __syncthreads();
  epi(GemmTile<TM, TN>{Ct, m0, n0, rt.Mr, rt.Nr, smem + TM * PB});
}
// Workgroup `bid` in [0, gemm_blocks(g)) of a GEMM: the virtual blocks bid, bid + grid, ... that carry
// runtime work.  A kernel may host several GEMMs by dispatching on block ranges.
template <class CFG, class AL, class BL, class EPI>
__device__ __forceinline__ void gemm_body(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part,
                                          int bid, float* smem) {
  const GemmRt rt = gemm_runtime<CFG>(g);
  const int tmr = (rt.Mr + CFG::TM - 1) / CFG::TM, tnr = (rt.Nr + CFG::TN - 1) / CFG::TN;
  const int per = (tmr * tnr * rt.Sr + 7) >> 3, grid = gemm_blocks(g);
  if constexpr (HasVec4<AL>::value || HasVec4<BL>::value) {
    if ((rt.Kr & 3) == 0 && rt.Kr >= 4 && vec_ok(al) && vec_ok(bl)) {
      for (int vb = bid; vb < 8 * per; vb += grid) {
        gemm_tile<CFG, true>(g, rt, al, bl, epi, part, vb, smem);
        __syncthreads();
      }
      return;
    }
  }
  for (int vb = bid; vb < 8 * per; vb += grid) {
    gemm_tile<CFG, false>(g, rt, al, bl, epi, part, vb, smem);
    __syncthreads();
  }
}

template <class CFG, class AL, class BL, class EPI>
__global__ void __launch_bounds__(256) gemm_kernel(GemmShape g, AL al, BL bl, EPI epi, float* part) {
  TGNX_STAMP(20);
  __shared__ __attribute__((aligned(16))) float smem[CFG::SMEM];
  gemm_body<CFG>(g, al, bl, epi, part, blockIdx.x, smem);
}

// Two independent GEMMs in one launch: blocks [0, gemm_blocks(g1)) run the first.
template <class C1, class C2, class AL1, class BL1, class EP1, class AL2, class BL2, class EP2>
__global__ void __launch_bounds__(256) gemm2_kernel(GemmShape g1, AL1 a1, BL1 b1, EP1 e1, float* p1, GemmShape g2,
                                                    AL2 a2, BL2 b2, EP2 e2, float* p2) {
  TGNX_STAMP(21);
  constexpr int SM = C1::SMEM > C2::SMEM ? C1::SMEM : C2::SMEM;
  __shared__ __attribute__((aligned(16))) float smem[SM];
  const int n1 = gemm_blocks(g1);
  if ((int)blockIdx.x < n1) gemm_body<C1>(g1, a1, b1, e1, p1, blockIdx.x, smem);
  else gemm_body<C2>(g2, a2, b2, e2, p2, blockIdx.x - n1, smem);
}

// Any number of independent GEMMs in one launch (block ranges in argument order; every GEMM range is a
// multiple of 8 blocks, so each GEMM keeps its XCD grouping when only GEMMs precede it).
template <class CFG, class AL, class BL, class EPI>
struct GemmJob {
  using Cfg = CFG;
  GemmShape g;
  AL al;
  BL bl;
  EPI epi;
  float* part;
};
template <class CFG, class AL, class BL, class EPI>
inline GemmJob<CFG, AL, BL, EPI> gemm_job(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part) {
  return GemmJob<CFG, AL, BL, EPI>{g, al, bl, epi, part};
}
template <class J>
__device__ __forceinline__ bool gemm_job_dispatch(const J& j, int& bid, float* smem) {
  const int nb = gemm_blocks(j.g);
  if (bid < nb) {
    gemm_body<typename J::Cfg>(j.g, j.al, j.bl, j.epi, j.part, bid, smem);
    return true;
  }
  bid -= nb;
  return false;
}
// a non-GEMM piece of work riding in a gemmN launch: nb 256-thread workgroups running f(bid, smem), smem
// at least SM floats of LDS (its block range unpadded: padding it to a multiple of the 8 XCDs measured ±0)
__host__ __device__ constexpr int blockjob_span(int nb) { return nb; }
template <class F, int SM = 4>
struct BlockJob {
  struct Cfg {
    static constexpr int SMEM = SM;
  };
  F f;
  int nb;
};
template <class F, int SM>
__device__ __forceinline__ bool gemm_job_dispatch(const BlockJob<F, SM>& j, int& bid, float* smem) {
  const int span = blockjob_span(j.nb);
  if (bid < span) {
    if (bid < j.nb) j.f(bid, smem);
    return true;
  }
  bid -= span;
  return false;
}
template <class J>
inline int job_blocks(const J& j) { return gemm_blocks(j.g); }
template <class F, int SM>
inline int job_blocks(const BlockJob<F, SM>& j) { return blockjob_span(j.nb); }
template <class... J>
#ifndef TGNX_GEMMN_WAVES
#define TGNX_GEMMN_WAVES 0  // amdgpu_waves_per_eu floor for gemmN launches (0 = compiler's choice; 5 measured +5 %)
#endif
#if TGNX_GEMMN_WAVES > 0
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TGNX_GEMMN_WAVES))) gemmN_kernel(J... j) {
#else
__global__ void __launch_bounds__(256) gemmN_kernel(J... j) {
#endif
  TGNX_STAMP(22);
  constexpr int SM = std::max({J::Cfg::SMEM...});
  __shared__ __attribute__((aligned(16))) float smem[SM];
  int bid = blockIdx.x;
  (void)(gemm_job_dispatch(j, bid, smem) || ...);
}
template <class... J>
static inline void gemmN_launch(hipStream_t s, const J&... j) {
  const int nb = (job_blocks(j) + ... + 0);
  if (nb > 0) launch_k(gemmN_kernel<J...>, dim3(nb), dim3(256), 0, s, j...);
}
// the same with a waves-per-SIMD floor for one launch (its register budget capped so W workgroups fit a CU)
template <int W, class... J>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) gemmN_kernel_w(J... j) {
  TGNX_STAMP(22);
  constexpr int SM = std::max({J::Cfg::SMEM...});
  __shared__ __attribute__((aligned(16))) float smem[SM];
  int bid = blockIdx.x;
  (void)(gemm_job_dispatch(j, bid, smem) || ...);
}
template <int W, class... J>
static inline void gemmN_launch_w(hipStream_t s, const J&... j) {
  const int nb = (job_blocks(j) + ... + 0);
  if constexpr (W > 0) {
    if (nb > 0) launch_k(gemmN_kernel_w<W, J...>, dim3(nb), dim3(256), 0, s, j...);
  } else {
    gemmN_launch(s, j...);
  }
}

// ---------------------------------------------------------------- split-K fixup
template <class CFG, class EPI>
struct GemmFix {
  GemmShape g;
  const float* part;
  EPI epi;
};
template <class CFG, class EPI>
inline GemmFix<CFG, EPI> gemm_fix(const GemmShape& g, const float* part, const EPI& epi) {
  return GemmFix<CFG, EPI>{g, part, epi};
}
// one output tile of a deferred GEMM: Σ partials over the runtime splits in order, then the epilogue
template <class CFG, class EPI>
__device__ void gemm_fix_tile(const GemmFix<CFG, EPI>& f, int tile, float* smem) {
  constexpr int TM = CFG::TM, TN = CFG::TN, FM = CFG::FM, FN = CFG::FN, PB = CFG::PB;
  const GemmRt rt = gemm_runtime<CFG>(f.g);
  const int tmi = tile / f.g.tiles_n, tni = tile % f.g.tiles_n;
  const int m0 = tmi * TM, n0 = tni * TN;
  if (m0 >= rt.Mr || n0 >= rt.Nr) return;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wr = (wv >> 1) * (TM / 2), wc = (wv & 1) * (TN / 2), li = lane & 15, lk = lane >> 4;
  float* Ct = smem;
  const GemmTile<TM, TN> tl{Ct, m0, n0, rt.Mr, rt.Nr, smem + TM * PB};
  auto sum_tile = [&]() {
    if constexpr (CFG::WS) {  // row-major partials
      constexpr int PER = TM * TN / 256, SU = 8;
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int x = threadIdx.x + 256 * e;
        float sum = 0.f;
        for (int q0 = 0; q0 < rt.Sr; q0 += SU) {
          float pv[SU];
#pragma unroll
          for (int u = 0; u < SU; ++u) pv[u] = f.part[((size_t)tile * f.g.S + min(q0 + u, rt.Sr - 1)) * TM * TN + x];
#pragma unroll
          for (int u = 0; u < SU; ++u) sum += pv[u] * f01(q0 + u < rt.Sr);
        }
        Ct[(x / TN) * PB + x % TN] = sum;
      }
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          // every split's partial in flight at once (clamped loads, masked sum; split order fixed)
          constexpr int SU = 8;
          f32x4_t sum = {0.f, 0.f, 0.f, 0.f};
          for (int q0 = 0; q0 < rt.Sr; q0 += SU) {
            f32x4_t pv[SU];
#pragma unroll
            for (int u = 0; u < SU; ++u) {
              const int q = min(q0 + u, rt.Sr - 1);
              pv[u] = reinterpret_cast<const f32x4_t*>(f.part + ((size_t)tile * f.g.S + q) * TM * TN)
                  [((wv * FM + i) * FN + j) * 64 + lane];
            }
#pragma unroll
            for (int u = 0; u < SU; ++u) sum += pv[u] * f01(q0 + u < rt.Sr);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) Ct[(wr + 16 * i + lk * 4 + r) * PB + wc + 16 * j + li] = sum[r];
        }
    }
  };
  sum_tile();
  __syncthreads();
  f.epi(tl);
}
template <class CFG, class EPI>
__device__ __forceinline__ bool gemm_fix_dispatch(const GemmFix<CFG, EPI>& f, int& bid, float* smem) {
  const int nt = f.g.tiles_m * f.g.tiles_n;
  if (bid < nt) {
    gemm_fix_tile(f, bid, smem);
    return true;
  }
  bid -= nt;
  return false;
}
template <class CFG, class EPI>
inline int gemm_fix_blocks(const GemmFix<CFG, EPI>& f) { return f.g.tiles_m * f.g.tiles_n; }

constexpr int GEMM_FIX_SMEM = 64 * 65 + 512;  // floats: the largest C tile (G64) + epilogue scratch

// Sum the partials of several deferred GEMMs (block ranges in argument order); the first `head` blocks
// and the blocks past the GEMMs call `tail(bid, smem)` (bid: 0 .. head - 1, then head, head + 1, ...):
// extra work that rides in the same launch, the head blocks dispatched first.
// XCD-contiguous tiles: the fix range is padded to a multiple of the 8 XCDs and XCD x takes
// the run [x nfix / 8, (x + 1) nfix / 8) of tiles in order, so the n-neighbour tiles of a weight row block run
// on one XCD.  A 32-float tile row of a weight whose row length is not a multiple of 32 floats (572 + 1, 272,
// 101, 100) straddles two 128-B lines shared with its neighbour tile; with bid-order tiles the neighbour ran on
// another XCD and every Adam operand line (param, m, v) left HBM twice.
template <class TAIL, class... F>
__global__ void __launch_bounds__(256) gemm_fixup_kernel(TAIL tail, int head, int nfix, F... f) {
  TGNX_STAMP(23);
  __shared__ __attribute__((aligned(16))) float smem[GEMM_FIX_SMEM];
  int bid = blockIdx.x;
  if (bid < head) {
    tail(bid, smem);
    return;
  }
  bid -= head;
  if (bid < nfix) {
    bid = (bid & 7) * (nfix >> 3) + (bid >> 3);
    (gemm_fix_dispatch(f, bid, smem) || ...);  // (padding blocks: past every GEMM's tiles)
    return;
  }
  tail(head + bid - nfix, smem);
}
template <class... F>
inline int gemm_fix_range(const F&... f) {
  const int nt = (gemm_fix_blocks(f) + ... + 0);
  return (nt + 7) & ~7;
}
struct NoTail {
  __device__ void operator()(int, float*) const {}
};

// Epilogue: C[m, n] = v (+ bias[n]) (+= C if accumulate), row-major ldc.
struct EpiStore {
  float* C;
  const float* bias;
  int ldc, accumulate;
  template <class T>
  __device__ void operator()(const T& t) const {
    float v[T::per];
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int r = T::row_of(i), cc = T::col_of(i), m = t.m0 + r, n = t.n0 + cc;
      const bool ok = m < t.M && n < t.N;
      v[i] = t(r, cc) + ((ok && bias) ? bias[n] : 0.f) + ((ok && accumulate) ? C[(int64_t)m * ldc + n] : 0.f);
    }
#pragma unroll
    for (int i = 0; i < T::per; ++i) {
      const int r = T::row_of(i), cc = T::col_of(i), m = t.m0 + r, n = t.n0 + cc;
      if (m < t.M && n < t.N) C[(int64_t)m * ldc + n] = v[i];
    }
  }
};

// epilogue of a deferred split-K job (its partials are summed and finished by gemm_fixup_kernel): never
// called, and keeps the finishing epilogue's fields out of the GEMM kernel's arguments
struct EpiDeferred {
  template <class T>
  __device__ void operator()(const T&) const {}
};

template <class CFG, class AL, class BL, class EPI>
static inline void gemm_launch(const GemmShape& g, const AL& al, const BL& bl, const EPI& epi, float* part,
                               hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return;
  launch_k(gemm_kernel<CFG, AL, BL, EPI>, dim3(gemm_blocks(g)), dim3(256), 0, s, g, al, bl, epi, part);
}
template <class C1, class C2, class AL1, class BL1, class EP1, class AL2, class BL2, class EP2>
static inline void gemm2_launch(const GemmShape& g1, const AL1& a1, const BL1& b1, const EP1& e1, float* p1,
                                const GemmShape& g2, const AL2& a2, const BL2& b2, const EP2& e2, float* p2,
                                hipStream_t s) {
  gemm2_kernel<C1, C2, AL1, BL1, EP1, AL2, BL2, EP2>
      <<<gemm_blocks(g1) + gemm_blocks(g2), 256, 0, s>>>(g1, a1, b1, e1, p1, g2, a2, b2, e2, p2);
}
template <class TAIL, class... F>
static inline void gemm_fixup_launch(int tail_blocks, const TAIL& tail, hipStream_t s, const F&... f) {
  const int nfix = gemm_fix_range(f...), nb = nfix + tail_blocks;
  if (nb > 0) launch_k(gemm_fixup_kernel<TAIL, F...>, dim3(nb), dim3(256), 0, s, tail, 0, nfix, f...);
}
// the same with `head` of the tail blocks first in the grid
template <class TAIL, class... F>
static inline void gemm_fixup_launch_h(int head, int tail_blocks, const TAIL& tail, hipStream_t s, const F&... f) {
  const int nfix = gemm_fix_range(f...), nb = nfix + tail_blocks;
  if (nb > 0) launch_k(gemm_fixup_kernel<TAIL, F...>, dim3(nb), dim3(256), 0, s, tail, head, nfix, f...);
}

}  // namespace tgnx
