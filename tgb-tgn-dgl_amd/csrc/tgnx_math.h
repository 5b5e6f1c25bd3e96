// Shared device math: exact-reduction sin/cos for time encodings and counter-based dropout masks.
#pragma once
#include "tgnx_common.h"

namespace tgnx {

// sin/cos of a float argument with an exact reduction: Cody-Waite in double (pi/2 split in two
// doubles, exact for |z| < 2^31) and double polynomials on |r| <= pi/4 (fdlibm kernel
// coefficients), rounded once to float.  Time-encoding arguments w*dt + b reach 1e6..1e9, where
// ocml's sincosf takes a long, divergent Payne-Hanek path; fp64 FMA runs at the fp32 rate on gfx950.
__device__ __forceinline__ void te_reduce(float z, double& r, int& q) {
  const double x = (double)z;
  const double k = rint(x * 0.63661977236758134308);
  r = fma(-k, 1.5707963267948965580e+00, x);
  r = fma(-k, 6.1232339957367658e-17, r);
  q = (int)(int64_t)k;
}
__device__ __forceinline__ double te_sin_poly(double r, double r2) {
  return r + r * r2 * (-1.66666666666666324348e-01 + r2 * (8.33333333332248946124e-03 +
         r2 * (-1.98412698298579493134e-04 + r2 * (2.75573137070700676789e-06 + r2 * -2.50507602534068634195e-08))));
}
__device__ __forceinline__ double te_cos_poly(double r2) {
  return 1.0 - 0.5 * r2 + r2 * r2 * (4.16666666666666019037e-02 + r2 * (-1.38888888888741095749e-03 +
         r2 * (2.48015872894767294178e-05 + r2 * (-2.75573143513906633035e-07 + r2 * 2.08757232129817482790e-09))));
}
__device__ __forceinline__ void te_sincos(float z, float& sn, float& cs) {
  double r; int q;
  te_reduce(z, r, q);
  const double r2 = r * r, s = te_sin_poly(r, r2), co = te_cos_poly(r2);
  const double s1 = (q & 1) ? co : s, c1 = (q & 1) ? s : co;
  sn = (float)((q & 2) ? -s1 : s1);
  cs = (float)(((q + 1) & 2) ? -c1 : c1);
}
__device__ __forceinline__ float te_cos(float z) {
  double r; int q;
  te_reduce(z, r, q);
  const double r2 = r * r;
  const double v = (q & 1) ? te_sin_poly(r, r2) : te_cos_poly(r2);
  return (float)(((q + 1) & 2) ? -v : v);
}


// Dropout masks: a 64-bit base per (batch seed, stream, key) computed once per edge / node, then
// a 32-bit murmur finaliser per element.  Forward and backward call the same functions, and
// duplicate (block, root) segments share keys, as the reference draws one mask per block.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_base(uint64_t seed, uint64_t stream, uint64_t key, uint64_t sub) {
  return (uint32_t)hash4(seed, stream, key, sub);
}
__device__ __forceinline__ float keep32(uint32_t base, uint32_t idx, float p, float inv) {
  const uint32_t h = fmix32(base ^ (idx * 0x9E3779B9u));
  // u = (h >> 8) 2^-24 >= p  <=>  (h >> 8) >= ceil(p 2^24) (both sides exact): an integer compare, its threshold
  // loop-invariant (p is a kernel argument)
  const uint32_t thr = (uint32_t)ceilf(p * 16777216.0f);
  return (h >> 8) >= thr ? inv : 0.0f;
}

}  // namespace tgnx
