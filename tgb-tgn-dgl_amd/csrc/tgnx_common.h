// Shared device/host helpers for libtgnx (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
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

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

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

// Sort n distinct uint64 keys in LDS, ascending, by the whole block: barrier-free rank sort
// (each key's slot = number of smaller keys) for n <= 1024, bitonic above.  `tmp` holds n keys.
__device__ __forceinline__ void sort_u64(uint64_t* key, uint64_t* tmp, int n, int n_pow2) {
  if (n <= 1024) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) tmp[i] = key[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const uint64_t k = tmp[i];
      int r = 0;
      for (int j = 0; j < n; ++j) r += tmp[j] < k;
      key[r] = k;
    }
    for (int i = n + threadIdx.x; i < n_pow2; i += blockDim.x) key[i] = ~0ull;
    __syncthreads();
  } else {
    bitonic_sort_u64(key, n_pow2);
  }
}

__host__ __device__ __forceinline__ int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace tgnx
