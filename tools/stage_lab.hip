// Staging lab (not part of libtgnx): how fast can a workgroup pull a small weight block (80 KB) into LDS
// when every workgroup of the grid reads the same block, vs distinct blocks, vs one workgroup, and
// with the block freshly written by the previous kernel (the step's parameter buffer is rewritten by
// the fused Adam of the previous step).  Per-workgroup durations from s_memrealtime.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/stage_lab.hip -o /tmp/stage_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int N4 = 5000;  // float4 per workgroup (80 KB)

// MODE 0: register staging, 256 threads, everything in flight (20 float4 per thread)
// MODE 1: register staging, 192 threads (waves 1-3), 27 float4 per thread
// MODE 2: LDS-DMA (global_load_lds 16 B), 256 threads
template <int MODE>
__global__ void __launch_bounds__(256) stage(const float4* src, int stride4, float* out, unsigned long long* dur) {
  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const float4* s = src + (size_t)blockIdx.x * stride4;
  const int tid = threadIdx.x;
  if (MODE == 0) {
    constexpr int U = (N4 + 255) / 256;
    float4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = s[min(tid + 256 * u, N4 - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (tid + 256 * u < N4) lds[tid + 256 * u] = r[u];
  } else if (MODE == 1) {
    if (tid >= 64) {
      constexpr int U = (N4 + 191) / 192;
      const int st = tid - 64;
      float4 r[U];
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = s[min(st + 192 * u, N4 - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (st + 192 * u < N4) lds[st + 192 * u] = r[u];
    }
  } else {
    const int wv = tid >> 6, lane = tid & 63;
    for (int b = wv * 64; b < N4; b += 256) {  // one 1 KB wave-instruction per 64 float4
      __builtin_amdgcn_global_load_lds((const void*)(s + min(b + lane, N4 - 1)), (__attribute__((address_space(3))) void*)(lds + b), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) dur[blockIdx.x] = t1 - t0;
  float acc = 0.f;
  for (int x = tid; x < N4; x += 256) acc += lds[x].x + lds[x].w;
  if (acc == 1234.5f) out[blockIdx.x] = acc;
}

__global__ void touch(float* p, int n) {  // rewrite the block (as Adam rewrites the parameters)
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) p[x] = p[x] * 1.0000001f;
}

int main() {
  const int G = 200;
  float* src;
  CK(hipMalloc(&src, (size_t)G * N4 * 16));
  CK(hipMemset(src, 0, (size_t)G * N4 * 16));
  float* out;
  CK(hipMalloc(&out, G * 4));
  unsigned long long* dur;
  CK(hipMalloc(&dur, G * 8));
  std::vector<unsigned long long> h(G);
  auto k0 = stage<0>;
  auto k1 = stage<1>;
  auto k2 = stage<2>;
  for (auto k : {k0, k1, k2}) CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  const char* names[3] = {"reg 256 thr", "reg 192 thr", "lds-dma"};
  for (int mode = 0; mode < 3; ++mode) {
    auto k = mode == 0 ? k0 : mode == 1 ? k1 : k2;
    for (int cfg = 0; cfg < 5; ++cfg) {
      // cfg 0: all WGs same block, warm; 1: same block, rewritten by the previous kernel; 2: distinct blocks,
      // warm; 3: distinct, rewritten; 4: one WG
      const int grid = cfg == 4 ? 1 : G;
      const int stride = (cfg == 2 || cfg == 3) ? N4 : 0;
      double avg = 0, mx = 0;
      for (int rep = 0; rep < 20; ++rep) {
        if (cfg == 1) touch<<<64, 256>>>(src, N4 * 4);
        if (cfg == 3) touch<<<1024, 256>>>(src, G * N4 * 4);
        k<<<grid, 256, N4 * 16>>>((const float4*)src, stride, out, dur);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), dur, grid * 8, hipMemcpyDeviceToHost));
        if (rep < 5) continue;
        double a = 0, m = 0;
        for (int b = 0; b < grid; ++b) {
          a += h[b] * 0.01;
          m = std::max(m, h[b] * 0.01);
        }
        avg += a / grid / 15;
        mx += m / 15;
      }
      const char* cn[5] = {"same block, warm", "same block, rewritten", "distinct, warm", "distinct, rewritten", "one WG"};
      printf("%-12s %-22s WG avg %6.2f us  max %6.2f us  (80 KB: %5.1f GB/s per WG avg)\n", names[mode], cn[cfg], avg, mx,
             80e3 / (avg * 1e3));
    }
  }
  return 0;
}
