// C ABI of the MFMA GEMM (tgnx_gemm.h): C = op(A) op(B) (+ bias) (+ C).
#include "tgnx_gemm.h"

using namespace tgnx;

// K <= 256: one workgroup per tile loops over K; larger K: split-K partials + a fixup launch
static GemmShape gemm_api_shape(int64_t M, int64_t N, int64_t K) {
  if (K <= 4 * GKC) return gemm_shape((int)M, (int)N, (int)K, GKC);
  return gemm_shape_split((int)M, (int)N, (int)K, GKC, nullptr, nullptr, nullptr, 32);
}

extern "C" {

size_t tgnx_gemm_f32_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 256;
  const GemmShape g = gemm_api_shape(M, N, K);
  return gemm_partial_floats(g) * 4 + 256;
}

int tgnx_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int32_t trans_a, const float* B,
                  int64_t ldb, int32_t trans_b, float* C, int64_t ldc, const float* bias, int32_t accumulate, void* ws,
                  size_t ws_bytes, void* stream) {
  TGNX_CHECK_ARG(M >= 0 && N >= 0 && K >= 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30),
                 "tgnx_gemm_f32: bad sizes");
  if (M == 0 || N == 0) return TGNX_OK;
  TGNX_CHECK_ARG(K > 0, "tgnx_gemm_f32: K must be positive");
  TGNX_CHECK_ARG(A && B && C && ws, "tgnx_gemm_f32: null pointer");
  TGNX_CHECK_ARG(ws_bytes >= tgnx_gemm_f32_ws_bytes(M, N, K), "tgnx_gemm_f32: workspace too small");
  const GemmShape g = gemm_api_shape(M, N, K);
  float* part = reinterpret_cast<float*>(ws);
  hipStream_t s = as_stream(stream);
  const int Kc = (int)K;
  // A element (m, k): trans_a ? A[k*lda + m] : A[m*lda + k];  B element (k, n): trans_b ? B[n*ldb + k] : B[k*ldb + n]
  EpiStore epi{C, bias, (int)ldc, accumulate};
  const float* Ap = A;
  const float* Bp = B;
  auto run = [&](const auto& al, const auto& bl) {
    gemm_launch(g, al, bl, epi, part, s);
    if (g.deferred) gemm_fixup_launch(0, NoTail{}, s, GemmFix<EpiStore>{g, part, epi});
  };
  if (!trans_a && trans_b)
    run(LoadRowK{Ap, (int)M, Kc, (int)lda}, LoadRowK{Bp, (int)N, Kc, (int)ldb});
  else if (!trans_a && !trans_b)
    run(LoadRowK{Ap, (int)M, Kc, (int)lda}, LoadKRow{Bp, (int)N, Kc, (int)ldb});
  else if (trans_a && trans_b)
    run(LoadKRow{Ap, (int)M, Kc, (int)lda}, LoadRowK{Bp, (int)N, Kc, (int)ldb});
  else
    run(LoadKRow{Ap, (int)M, Kc, (int)lda}, LoadKRow{Bp, (int)N, Kc, (int)ldb});
  TGNX_LAUNCH_CHECK("tgnx_gemm_f32");
  return TGNX_OK;
}

}  // extern "C"
