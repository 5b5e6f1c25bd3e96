// Sort lab (not part of libtgnx): one 1024-thread workgroup sorting the 2B = 400 distinct keys of a
// ring / store plan with the library's sorts, timed inside the kernel with s_memrealtime (100 MHz) and
// s_memtime (shader clock), so the effective clock shows too.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I tgb-tgn-dgl_amd/csrc tools/sort_lab.hip -o lab/sort_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tgnx_common.h"

namespace tgnx {
void set_error(const char*, ...) {}
}
using namespace tgnx;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int MODE>
__global__ void __launch_bounds__(1024) sortk(const uint64_t* in, uint64_t* out, int n, unsigned long long* t) {
  __shared__ uint64_t key[1024], tmp[1024];
  for (int i = threadIdx.x; i < n; i += blockDim.x) key[i] = in[i];
  __syncthreads();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  const int np = next_pow2(n);
  if (MODE == 0) sort_u64(key, tmp, n, np, true);   // rank sort
  else if (MODE == 1) sort_u64(key, tmp, n, np, false);  // register bitonic
  else {  // empty: barrier cost only
    __syncthreads();
  }
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = key[i];
  if (threadIdx.x == 0) {
    t[0] = r1 - r0;
    t[1] = c1 - c0;
  }
}

int main() {
  const int n = 400;
  std::vector<uint64_t> h(n);
  srand(3);
  for (int i = 0; i < n; ++i) h[i] = ((uint64_t)(rand() % 9227) << 32) | ((uint64_t)(n - 1 - i) << 1) | (i & 1);
  uint64_t *in, *out;
  unsigned long long* t;
  CK(hipMalloc(&in, n * 8));
  CK(hipMalloc(&out, n * 8));
  CK(hipMalloc(&t, 16));
  CK(hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice));
  const char* names[3] = {"rank sort", "register bitonic", "barrier only"};
  for (int mode = 0; mode < 3; ++mode) {
    double rs = 0, cs = 0;
    for (int rep = 0; rep < 30; ++rep) {
      if (mode == 0) sortk<0><<<1, 1024>>>(in, out, n, t);
      else if (mode == 1) sortk<1><<<1, 1024>>>(in, out, n, t);
      else sortk<2><<<1, 1024>>>(in, out, n, t);
      CK(hipDeviceSynchronize());
      unsigned long long ht[2];
      CK(hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost));
      if (rep >= 10) {
        rs += ht[0] * 0.01 / 20;
        cs += ht[1] / 20.0;
      }
    }
    std::vector<uint64_t> o(n);
    CK(hipMemcpy(o.data(), out, n * 8, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int i = 1; i < n; ++i) ok &= o[i - 1] < o[i];
    printf("%-18s %6.2f us  %8.0f shader clocks  (%.2f GHz)  sorted %d\n", names[mode], rs, cs, cs / rs / 1e3, ok);
  }
  return 0;
}
