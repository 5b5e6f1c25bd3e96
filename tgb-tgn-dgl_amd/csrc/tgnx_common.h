// Shared device/host helpers for libtgnx (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/tgnx.h"

namespace tgnx {

constexpr int WAVE = 64;

// ---------------------------------------------------------------- error plumbing
void set_error(const char* fmt, ...);

#define TGNX_CHECK_ARG(cond, ...)                          \
  do {                                                     \
    if (!(cond)) {                                         \
      ::tgnx::set_error(__VA_ARGS__);                      \
      return TGNX_EINVAL;                                  \
    }                                                      \
  } while (0)

#define TGNX_LAUNCH_CHECK(name)                                                  \
  do {                                                                           \
    hipError_t _e = hipGetLastError();                                           \
    if (_e != hipSuccess) {                                                      \
      ::tgnx::set_error("%s: launch failed: %s", name, hipGetErrorString(_e));   \
      return TGNX_EHIP;                                                          \
    }                                                                            \
  } while (0)

#define TGNX_HIP_CHECK(call)                                                     \
  do {                                                                           \
    hipError_t _e = (call);                                                      \
    if (_e != hipSuccess) {                                                      \
      ::tgnx::set_error("%s: %s", #call, hipGetErrorString(_e));                 \
      return TGNX_EHIP;                                                          \
    }                                                                            \
  } while (0)

// kernel probe (tgnx_host.cpp): inside an open probe region, the first launch through launch_k binds the
// probe's kernel event pair to itself (hipExtLaunchKernelGGL start / stop events = the dispatch's own begin /
// end timestamps); every other launch is a plain one.
bool probe_take(hipEvent_t* k0, hipEvent_t* k1);
template <typename... KArgs, typename... Args>
inline void launch_k(void (*kern)(KArgs...), dim3 grid, dim3 block, uint32_t smem, hipStream_t s, Args... args) {
  hipEvent_t k0, k1;
  if (probe_take(&k0, &k1))
    hipExtLaunchKernelGGL(kern, grid, block, smem, s, k0, k1, 0, args...);
  else
    hipLaunchKernelGGL(kern, grid, block, smem, s, args...);
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- wave timeline stamps (diagnostic build)
// Built with -DTGNX_STAMPS: every instrumented kernel's waves record {start, end} (s_memrealtime, 100 MHz),
// the kernel id, block and XCC into a buffer set by tgnx_stamps_set (tools/stamps.py reads it).  Without the
// flag TGNX_STAMP(k) is empty and the buffer entry points return TGNX_EINVAL.
#ifdef TGNX_STAMPS
#ifndef TGNX_STAMP_TID
#define TGNX_STAMP_TID 0  // the recording thread (its wave's view of the checkpoints)
#endif
struct StampRec {
  unsigned long long t0, t1;
  unsigned kid, blk, xcc, wave;
};
static __device__ StampRec* g_stamp_buf;
static __device__ unsigned g_stamp_cap;             // records per shard
static __device__ unsigned g_stamp_cnt[64 * 32];    // 64 shards (by block), one 128-B line each
struct StampScope {  // wave 0 of each workgroup records
  unsigned long long t0;
  unsigned kid, mid = 0;  // two checkpoints: ticks since t0 (16 bits each) at TGNX_STAMP_AT(0 / 1)
  __device__ explicit StampScope(unsigned k) : t0(__builtin_amdgcn_s_memrealtime()), kid(k) {}
  __device__ void at(int slot) {
    const unsigned d = (unsigned)min(__builtin_amdgcn_s_memrealtime() - t0, 0xFFFFull);
    mid = slot ? (mid & 0xFFFFu) | (d << 16) : (mid & 0xFFFF0000u) | d;
  }
  __device__ ~StampScope() {
    if (threadIdx.x == TGNX_STAMP_TID && g_stamp_buf) {
      const unsigned sh = blockIdx.x & 63, i = atomicAdd(&g_stamp_cnt[sh * 32], 1u);
      if (i < g_stamp_cap)
        g_stamp_buf[(size_t)sh * g_stamp_cap + i] =
            StampRec{t0, __builtin_amdgcn_s_memrealtime(), kid, blockIdx.x,
                     (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20), mid};
    }
  }
};
#define TGNX_STAMP(k) ::tgnx::StampScope tgnx_stamp_scope_(k)
#define TGNX_STAMP_AT(slot) tgnx_stamp_scope_.at(slot)
#else
#define TGNX_STAMP(k)
#define TGNX_STAMP_AT(slot)
#endif

// ---------------------------------------------------------------- counter-based RNG
// splitmix64 finaliser: statistically strong, stateless, identical in every replay.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t hash4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return mix64(a ^ mix64(b ^ mix64(c ^ mix64(d))));
}
// uniform in [0,1) with 24 bits
__device__ __forceinline__ float u01(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------- wave / block primitives
__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
  return v;
}
// Full-wave reductions on DPP / permlane swaps: no LDS round trip (__shfl_xor lowers to ds_bpermute).
// Every lane of the wave must be active; every lane gets the same (bitwise) result.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float swap16_sum(float v) {  // v + v[lane ^ 16]
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}
__device__ __forceinline__ float swap32_sum(float v) {  // v + v[lane ^ 32]
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}
__device__ __forceinline__ float wave_sum_f(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of the 8-lane half-row (quads are uniform)
  v += dpp_f<0x140>(v);  // row_mirror: the other half of the 16-lane row
  return swap32_sum(swap16_sum(v));
}
// sum over each 32-lane half (lanes 0-31 and 32-63 get their own half's sum)
__device__ __forceinline__ float half_sum_f(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return swap16_sum(v);
}
__device__ __forceinline__ float wave_max_f(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = fmaxf(__int_as_float(p[0]), __int_as_float(p[1]));
  p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(p[0]), __int_as_float(p[1]));
}
__device__ __forceinline__ int wave_min_i(int v) {
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));
  auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = min((int)p[0], (int)p[1]);
  p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return min((int)p[0], (int)p[1]);
}
// v of lane ^ 32 / lane ^ 16 (exchanges through the permlane swaps; full wave)
__device__ __forceinline__ float xor32_f(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float((threadIdx.x & 32) ? p[0] : p[1]);
}
__device__ __forceinline__ float xor16_f(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float((threadIdx.x & 16) ? p[0] : p[1]);
}
// lane l (wave-uniform) of v, through a scalar register
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int lane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int wave_incl_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    int u = __shfl_up(v, o, WAVE);
    if (l >= o) v += u;
  }
  return v;
}

// Exclusive scan over one value per thread of a whole workgroup (<= 1024 threads).
// `sh` must hold >= 16 ints of LDS. Returns the exclusive prefix; *total gets the sum.
__device__ __forceinline__ int block_excl_scan(int v, int* sh, int* total) {
  const int l = lane_id();
  const int w = threadIdx.x / WAVE;
  const int nw = (blockDim.x + WAVE - 1) / WAVE;
  int inc = wave_incl_scan(v);
  if (l == WAVE - 1) sh[w] = inc;
  __syncthreads();
  if (w == 0) {
    int s = (l < nw) ? sh[l] : 0;
    int si = wave_incl_scan(s);
    if (l < nw) sh[l] = si - s;
    if (l == nw - 1) sh[16] = si;
  }
  __syncthreads();
  int r = inc - v + sh[w];
  *total = sh[16];
  __syncthreads();
  return r;
}

// Two exclusive scans sharing the barriers of one.  `sh` must hold >= 40 ints of LDS.
__device__ __forceinline__ void block_excl_scan2(int a, int b, int* sh, int* ra, int* rb, int* ta, int* tb) {
  const int l = lane_id();
  const int w = threadIdx.x / WAVE;
  const int nw = (blockDim.x + WAVE - 1) / WAVE;
  const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
  if (l == WAVE - 1) {
    sh[w] = ia;
    sh[20 + w] = ib;
  }
  __syncthreads();
  if (w == 0) {
    const int s = (l < nw) ? sh[l] : 0, t = (l < nw) ? sh[20 + l] : 0;
    const int si = wave_incl_scan(s), ti = wave_incl_scan(t);
    if (l < nw) {
      sh[l] = si - s;
      sh[20 + l] = ti - t;
    }
    if (l == nw - 1) {
      sh[16] = si;
      sh[36] = ti;
    }
  }
  __syncthreads();
  *ra = ia - a + sh[w];
  *rb = ib - b + sh[20 + w];
  *ta = sh[16];
  *tb = sh[36];
  __syncthreads();
}

// In-LDS bitonic sort of n (power of two) uint64 keys, ascending, by the whole block.
__device__ __forceinline__ void bitonic_sort_u64(uint64_t* key, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int ixj = i ^ j;
        if (ixj > i) {
          uint64_t a = key[i], b = key[ixj];
          bool up = (i & k) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const unsigned lo = __shfl_xor((unsigned)v, m, WAVE), hi = __shfl_xor((unsigned)(v >> 32), m, WAVE);
  return ((uint64_t)hi << 32) | lo;
}

// lane i <- lane i ^ J, picking the cheapest cross-lane path for each distance: DPP quad_perm
// (1, 2), DPP row_ror:8 (8), ds_swizzle xor mode within 32 lanes (4), v_permlane16_swap (16) and
// v_permlane32_swap (32) (full waves; the round-2 shuffles, ds_bpermute LDS round trips, measured 3.7 % slower).
template <int J>
__device__ __forceinline__ unsigned xlane_xor(unsigned v) {
  if constexpr (J == 1) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (J == 2) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (J == 8) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
  else if constexpr (J == 16) {  // v_permlane16_swap: rows 0 <-> 1, 2 <-> 3
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (threadIdx.x & 16) ? (unsigned)p[0] : (unsigned)p[1];
  } else if constexpr (J == 32) {  // v_permlane32_swap: halves
    const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (threadIdx.x & 32) ? (unsigned)p[0] : (unsigned)p[1];
  }
  else if constexpr (J < 32) return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (J << 10));
  else return __shfl_xor(v, J, WAVE);
}
template <int J>
__device__ __forceinline__ uint64_t bitonic_lane_stage(uint64_t v, int i, int k) {
  const unsigned lo = xlane_xor<J>((unsigned)v), hi = xlane_xor<J>((unsigned)(v >> 32));
  const uint64_t o = ((uint64_t)hi << 32) | lo;
  const bool take_min = ((i & J) == 0) == ((i & k) == 0);
  return take_min ? (o < v ? o : v) : (o > v ? o : v);
}

// Bitonic sort of n (power of two, n <= blockDim.x) uint64 keys, ascending, one key per thread in
// registers: partner distances < 64 exchange across lanes (no barrier), larger ones through LDS,
// ping-ponging between `key` and `tmp` so each such stage needs a single barrier.
// For n = 1024: 45 cross-lane stages, 10 LDS stages.  Result in key[0, n).
__device__ __forceinline__ void sort_u64_reg(uint64_t* key, uint64_t* tmp, int n) {
  const int i = threadIdx.x;
  uint64_t v = i < n ? key[i] : ~0ull;
  const int wn = (n + WAVE - 1) & ~(WAVE - 1);  // whole waves holding keys
  int flip = 0;
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j >= WAVE; j >>= 1) {
      uint64_t* buf = flip ? tmp : key;
      flip ^= 1;
      if (i < n) buf[i] = v;
      __syncthreads();
      const uint64_t o = i < n ? buf[i ^ j] : v;
      const bool take_min = ((i & j) == 0) == ((i & k) == 0);
      v = take_min ? (o < v ? o : v) : (o > v ? o : v);
    }
    if (i < wn)  // waves past the keys skip the lane stages (a 1024-thread block sorting 512 keys)
      switch (k >= 64 ? 32 : k >> 1) {  // remaining distances 32..1 (wave-uniform)
        case 32: v = bitonic_lane_stage<32>(v, i, k); [[fallthrough]];
        case 16: v = bitonic_lane_stage<16>(v, i, k); [[fallthrough]];
        case 8: v = bitonic_lane_stage<8>(v, i, k); [[fallthrough]];
        case 4: v = bitonic_lane_stage<4>(v, i, k); [[fallthrough]];
        case 2: v = bitonic_lane_stage<2>(v, i, k); [[fallthrough]];
        default: v = bitonic_lane_stage<1>(v, i, k);
      }
  }
  __syncthreads();
  if (i < n) key[i] = v;
  __syncthreads();
}

// Rank sort of n DISTINCT uint64 keys (n <= blockDim.x): key i goes to position #{j : key[j] < key[i]}.
// Two threads per key when the block has them (adjacent lanes, each counting half the keys from LDS
// broadcast reads, 2 keys per ds_read_b128).  n^2 compares, but no dependent stages: 400 keys (a
// B = 200 ring / store plan) take ~1 us against ~5.5 us for the 39 lane + 6 LDS stages of the bitonic
// network (stamps timeline).  `tmp` holds n keys; the result is in key[0, n).
__device__ __forceinline__ void sort_u64_rank(uint64_t* key, uint64_t* tmp, int n) {
  const int P = 2 * n <= (int)blockDim.x ? 2 : 1;
  const int i = threadIdx.x / P, h = threadIdx.x % P;
  const int half = ((n + 3) >> 2) << 1;  // even split point (16-B aligned pairs)
  if (i < n) {
    const uint64_t v = key[i];
    const int j0 = P == 2 ? h * half : 0, j1 = P == 2 ? (h ? n : min(half, n)) : n;
    // 16 keys (8 ds_read_b128) in flight per round: a read-use chain per key pair waited the LDS latency
    // (~6.5 us for 400 keys, stamps timeline)
    int r = 0;
    int j = j0;
    for (; j + 15 < j1; j += 16) {
      uint64_t a[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) a[u] = key[j + u];
#pragma unroll
      for (int u = 0; u < 16; ++u) r += a[u] < v;
    }
    for (; j < j1; ++j) r += key[j] < v;
    if (P == 2) r += __shfl_xor(r, 1, WAVE);
    if (h == 0) tmp[r] = v;
  }
  __syncthreads();
  for (int x = threadIdx.x; x < n; x += blockDim.x) key[x] = tmp[x];
  __syncthreads();
}

// Sort of 64 < n <= 1024 DISTINCT keys in O(n log n) LDS work: each wave sorts 64-key chunks in
// registers (bitonic lane stages, no barriers), then each key's final position = its place in its chunk
// + a 7-step binary search (count of smaller keys) in every other chunk — independent searches, so
// their LDS latencies overlap.  The n^2 rank sort's compares made a 400-key plan VALU-bound (~5 us
// at 1024 threads, ~6.4 us at 256; stamps timeline).  tmp: roundup(n, 64) keys; result in key[0, n).
__device__ __forceinline__ uint64_t wave_sort64(uint64_t v, int lane) {
  for (int k = 2; k <= WAVE; k <<= 1) switch (k >> 1) {
      case 32: v = bitonic_lane_stage<32>(v, lane, k); [[fallthrough]];
      case 16: v = bitonic_lane_stage<16>(v, lane, k); [[fallthrough]];
      case 8: v = bitonic_lane_stage<8>(v, lane, k); [[fallthrough]];
      case 4: v = bitonic_lane_stage<4>(v, lane, k); [[fallthrough]];
      case 2: v = bitonic_lane_stage<2>(v, lane, k); [[fallthrough]];
      default: v = bitonic_lane_stage<1>(v, lane, k);
    }
  return v;
}
__device__ __forceinline__ void sort_u64_chunks(uint64_t* key, uint64_t* tmp, int n) {
  const int T = blockDim.x, t = threadIdx.x, lane = t & (WAVE - 1);
  const int C = (n + WAVE - 1) / WAVE;  // <= 16
  for (int ch = t / WAVE; ch < C; ch += T / WAVE) {
    const int p = ch * WAVE + lane;
    tmp[p] = wave_sort64(p < n ? key[p] : ~0ull, lane);
  }
  __syncthreads();
  // level-major in groups of four chunks: one search step of each of the four per round (independent LDS
  // reads in flight), 7 dependent rounds + the final compare per group.  The key's own chunk is searched too
  // (no per-thread branch): its count of smaller keys is the key's place in the chunk.  Chunk-major searches
  // with a divergent `ch == own` skip ran as 42 dependent LDS round trips per key at 400 keys (6.8 us at
  // 256 threads); sixteen chunks at once spilled to scratch.  Chunks past C are clamped and masked out.
  for (int p = t; p < n; p += T) {
    const uint64_t v = tmp[p];
    int r = 0;
    for (int g = 0; g < C; g += 4) {  // (uniform)
      const uint64_t* b0 = tmp + g * WAVE;
      const uint64_t* b1 = tmp + min(g + 1, C - 1) * WAVE;
      const uint64_t* b2 = tmp + min(g + 2, C - 1) * WAVE;
      const uint64_t* b3 = tmp + min(g + 3, C - 1) * WAVE;
      int q0 = 0, q1 = 0, q2 = 0, q3 = 0;
#pragma unroll
      for (int st = 32; st >= 1; st >>= 1) {
        const uint64_t o0 = b0[q0 + st - 1], o1 = b1[q1 + st - 1], o2 = b2[q2 + st - 1], o3 = b3[q3 + st - 1];
        q0 += o0 < v ? st : 0;
        q1 += o1 < v ? st : 0;
        q2 += o2 < v ? st : 0;
        q3 += o3 < v ? st : 0;
      }
      q0 += b0[q0] < v ? 1 : 0;
      q1 += b1[q1] < v ? 1 : 0;
      q2 += b2[q2] < v ? 1 : 0;
      q3 += b3[q3] < v ? 1 : 0;
      r += q0 + (g + 1 < C ? q1 : 0) + (g + 2 < C ? q2 : 0) + (g + 3 < C ? q3 : 0);
    }
    key[r] = v;
  }
  __syncthreads();
}

// Sort n uint64 keys in LDS, ascending, by the whole block (key[n, n_pow2) padded with ~0 on
// return): register bitonic when n_pow2 <= blockDim.x (`tmp` holds n_pow2 keys), LDS bitonic above.
// `distinct`: the keys are pairwise distinct and n <= blockDim.x -> rank sort.
// Bitonic sort of n (power of two, T < n <= 4 T with T = blockDim.x, a multiple of 64) uint64 keys with
// four keys per thread in registers (positions t, t + T, t + 2T, t + 3T): partner distances >= T are
// compare-exchanges inside the thread, 64 <= j < T one LDS round (ping-pong `key` / `tmp`, one barrier
// for all four registers), j < 64 cross-lane.  n = 4096 at T = 1024: 18 barriers instead of the 78 of
// bitonic_sort_u64 (3,200 keys: a data-parallel step's global-batch insert plan at world 8).  tmp: n keys.
#ifndef TGNX_SORT_CHUNKS_MIN
#define TGNX_SORT_CHUNKS_MIN 64  // distinct keys: chunked sort above this many (rank sort below)
#endif
__device__ __forceinline__ void cmpx_u64(uint64_t& a, uint64_t& b, bool up) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = up ? lo : hi;
  b = up ? hi : lo;
}
__device__ __forceinline__ void sort_u64_reg4(uint64_t* key, uint64_t* tmp, int n) {
  const int T = blockDim.x, t = threadIdx.x;
  const int nm = n / T;  // 2 or 4 registers in use
  uint64_t v[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) v[m] = m < nm ? key[t + m * T] : ~0ull;
  int flip = 0;
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j >= WAVE; j >>= 1) {
      if (j >= T) {  // same thread: register m pairs with m ^ (j / T)
        if (j == T) {
          cmpx_u64(v[0], v[1], (t & k) == 0);
          if (nm == 4) cmpx_u64(v[2], v[3], ((t + 2 * T) & k) == 0);
        } else {  // j == 2T
          cmpx_u64(v[0], v[2], (t & k) == 0);
          cmpx_u64(v[1], v[3], ((t + T) & k) == 0);
        }
        continue;
      }
      uint64_t* buf = flip ? tmp : key;
      flip ^= 1;
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (m < nm) buf[t + m * T] = v[m];
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 4; ++m)
        if (m < nm) {
          const int p = t + m * T;
          const uint64_t o = buf[p ^ j];
          const bool take_min = ((p & j) == 0) == ((p & k) == 0);
          v[m] = take_min ? (o < v[m] ? o : v[m]) : (o > v[m] ? o : v[m]);
        }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (m >= nm) continue;
      const int p = t + m * T;
      switch (k >= 64 ? 32 : k >> 1) {  // remaining distances 32..1
        case 32: v[m] = bitonic_lane_stage<32>(v[m], p, k); [[fallthrough]];
        case 16: v[m] = bitonic_lane_stage<16>(v[m], p, k); [[fallthrough]];
        case 8: v[m] = bitonic_lane_stage<8>(v[m], p, k); [[fallthrough]];
        case 4: v[m] = bitonic_lane_stage<4>(v[m], p, k); [[fallthrough]];
        case 2: v[m] = bitonic_lane_stage<2>(v[m], p, k); [[fallthrough]];
        default: v[m] = bitonic_lane_stage<1>(v[m], p, k);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < 4; ++m)
    if (m < nm) key[t + m * T] = v[m];
  __syncthreads();
}
// tmp_full: tmp holds n_pow2 keys (enables the four-keys-per-thread sort for T < n_pow2 <= 4 T)
__device__ __forceinline__ void sort_u64(uint64_t* key, uint64_t* tmp, int n, int n_pow2, bool distinct = false,
                                         bool tmp_full = false) {
  if (distinct && (n <= (int)blockDim.x || n <= 1024)) {
    if (n > TGNX_SORT_CHUNKS_MIN && n <= 1024) sort_u64_chunks(key, tmp, n);
    else sort_u64_rank(key, tmp, n);
    for (int i = n + threadIdx.x; i < n_pow2; i += blockDim.x) key[i] = ~0ull;
    __syncthreads();
    return;
  }
  for (int i = n + threadIdx.x; i < n_pow2; i += blockDim.x) key[i] = ~0ull;
  __syncthreads();
  if (n_pow2 <= (int)blockDim.x) sort_u64_reg(key, tmp, n_pow2);
  else if (tmp_full && n_pow2 <= 4 * (int)blockDim.x) sort_u64_reg4(key, tmp, n_pow2);
  else bitonic_sort_u64(key, n_pow2);
}

__host__ __device__ __forceinline__ int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace tgnx
