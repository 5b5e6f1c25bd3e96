// PMC calibration: kernels with a known byte count per access pattern, so the FETCH_SIZE / WRITE_SIZE (and raw
// TCC_EA0 request) counters of the TGN kernels can be read as bytes.  MI355X_MICROARCH.md (HBM section) pins
// only the 16-B-per-lane streaming read (FETCH_SIZE = half its bytes) and 16-B / atomic writes; every other
// width is "uncalibrated: calibrate on a known byte count in your own access pattern".  The TGN GEMM loaders
// read 4 B per lane (r-fast operands), 16 B per lane (vec4 k-fast operands) and 400-B gathered rows (memory
// rows, D = 100); the patterns below are those.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d out -o run -- tools/pmc_calib      (one counter group per pass)
// Every kernel touches each byte of its 64 MiB range once (rows: a random permutation of 400-B rows), except
// rd_line4 (one float per 128-B line: 4 B used, 128 B line), which shows the request granularity.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr size_t BYTES = 64ull << 20;
constexpr int NB = 2048, NT = 256;

__device__ __forceinline__ void sink(float* out, float v) {
  // one vector store per workgroup (keeps the loads live)
  __shared__ float red[NT / 64];
  for (int o = 32; o; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void rd_b128(const float4* p, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)NB * NT) {
    const float4 v = p[i];
    s += v.x + v.y + v.z + v.w;
  }
  sink(out, s);
}
__global__ void rd_b64(const float2* p, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)NB * NT) {
    const float2 v = p[i];
    s += v.x + v.y;
  }
  sink(out, s);
}
__global__ void rd_b32(const float* p, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)NB * NT) s += p[i];
  sink(out, s);
}
// one 400-B row (100 floats) per wave, rows in a random order: lanes 0..63 take floats lane and lane + 64
__global__ void rd_rows400(const float* p, const int* perm, int rows, float* out) {
  float s = 0.f;
  const int w = (blockIdx.x * NT + threadIdx.x) >> 6, lane = threadIdx.x & 63, nw = NB * NT / 64;
  for (int r = w; r < rows; r += nw) {
    const float* row = p + (size_t)perm[r] * 100;
    s += row[lane];
    if (lane < 36) s += row[64 + lane];
  }
  sink(out, s);
}
// one float per 128-B line, lines in a random order
__global__ void rd_line4(const float* p, const int* perm, int lines, float* out) {
  float s = 0.f;
  for (int i = blockIdx.x * NT + threadIdx.x; i < lines; i += NB * NT) s += p[(size_t)perm[i] * 32];
  sink(out, s);
}
__global__ void wr_b128(float4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)NB * NT) p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void wr_b32(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)NT + threadIdx.x; i < n; i += (size_t)NB * NT) p[i] = (float)i;
}
// one 400-B row per wave, random order (the memory-row / gradient-row stores)
__global__ void wr_rows400(float* p, const int* perm, int rows) {
  const int w = (blockIdx.x * NT + threadIdx.x) >> 6, lane = threadIdx.x & 63, nw = NB * NT / 64;
  for (int r = w; r < rows; r += nw) {
    float* row = p + (size_t)perm[r] * 100;
    row[lane] = (float)r;
    if (lane < 36) row[64 + lane] = (float)r;
  }
}

int main() {
  float *a, *b, *out;
  int *prow, *pline;
  const int rows = (int)(BYTES / 400), lines = (int)(BYTES / 128);
  CK(hipMalloc(&a, BYTES));
  CK(hipMalloc(&b, BYTES));
  CK(hipMalloc(&out, NB * sizeof(float)));
  CK(hipMalloc(&prow, rows * sizeof(int)));
  CK(hipMalloc(&pline, lines * sizeof(int)));
  std::mt19937 rng(7);
  std::vector<int> h(lines);
  std::iota(h.begin(), h.begin() + rows, 0);
  std::shuffle(h.begin(), h.begin() + rows, rng);
  CK(hipMemcpy(prow, h.data(), rows * sizeof(int), hipMemcpyHostToDevice));
  std::iota(h.begin(), h.end(), 0);
  std::shuffle(h.begin(), h.end(), rng);
  CK(hipMemcpy(pline, h.data(), lines * sizeof(int), hipMemcpyHostToDevice));
  CK(hipMemset(a, 0, BYTES));
  CK(hipMemset(b, 0, BYTES));
  const size_t n = BYTES / 4;
  for (int rep = 0; rep < 3; ++rep) {  // a and b alternate so no kernel starts on its own L2-resident range
    rd_b128<<<NB, NT>>>((const float4*)a, n / 4, out);
    rd_b64<<<NB, NT>>>((const float2*)b, n / 2, out);
    rd_b32<<<NB, NT>>>(a, n, out);
    rd_rows400<<<NB, NT>>>(b, prow, rows, out);
    rd_line4<<<NB, NT>>>(a, pline, lines, out);
    wr_b128<<<NB, NT>>>((float4*)b, n / 4);
    wr_b32<<<NB, NT>>>(a, n);
    wr_rows400<<<NB, NT>>>(b, prow, rows);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::printf("{\"bytes\": %zu, \"rows400\": %d, \"lines128\": %d, \"rd_line4_used_bytes\": %zu}\n", BYTES, rows, lines,
              (size_t)lines * 4);
  return 0;
}
