// C ABI of the MFMA GEMM (tgnx_gemm.h): C = op(A) op(B) (+ bias) (+ C).
#include "tgnx_gemm.h"

using namespace tgnx;

// Tile config: 64x64 once that already fills the chip, else 16x16 wave-split tiles with direct operands (the
// TGN step's long-K config, GemmCfg::DR: this entry point is also its unit test against torch).  K up to 4
// chunks: one workgroup per tile loops over K; larger K: split-K partials + a fixup launch.
static bool api_big(int64_t M, int64_t N) { return ((M + 63) / 64) * ((N + 63) / 64) >= 512; }
using GD = GemmCfg<16, 16, 64, 1, true, 3>;
template <class CFG>
static GemmShape gemm_api_shape(int64_t M, int64_t N, int64_t K) {
  if (K <= 4 * CFG::KC) return gemm_shape<CFG>((int)M, (int)N, (int)K);
  return gemm_shape_split<CFG>((int)M, (int)N, (int)K, nullptr, nullptr, nullptr, 16);
}

extern "C" {

size_t tgnx_gemm_f32_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 256;
  const GemmShape g = api_big(M, N) ? gemm_api_shape<G64>(M, N, K) : gemm_api_shape<GD>(M, N, K);
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
  float* part = reinterpret_cast<float*>(ws);
  hipStream_t s = as_stream(stream);
  const int Kc = (int)K;
  // A element (m, k): trans_a ? A[k*lda + m] : A[m*lda + k];  B element (k, n): trans_b ? B[n*ldb + k] : B[k*ldb + n]
  EpiStore epi{C, bias, (int)ldc, accumulate};
  auto run2 = [&](auto cfg, const auto& al, const auto& bl) {
    using CFG = decltype(cfg);
    const GemmShape g = gemm_api_shape<CFG>(M, N, K);
    gemm_launch<CFG>(g, al, bl, epi, part, s);
    if (g.deferred) gemm_fixup_launch(0, NoTail{}, s, gemm_fix<CFG>(g, part, epi));
  };
  auto run = [&](const auto& al, const auto& bl) {
    if (api_big(M, N)) run2(G64{}, al, bl);
    else run2(GD{}, al, bl);
  };
  if (!trans_a && trans_b)
    run(LoadRowK{A, (int)M, Kc, (int)lda}, LoadRowK{B, (int)N, Kc, (int)ldb});
  else if (!trans_a && !trans_b)
    run(LoadRowK{A, (int)M, Kc, (int)lda}, LoadKRow{B, (int)N, Kc, (int)ldb});
  else if (trans_a && trans_b)
    run(LoadKRow{A, (int)M, Kc, (int)lda}, LoadRowK{B, (int)N, Kc, (int)ldb});
  else
    run(LoadKRow{A, (int)M, Kc, (int)lda}, LoadKRow{B, (int)N, Kc, (int)ldb});
  TGNX_LAUNCH_CHECK("tgnx_gemm_f32");
  return TGNX_OK;
}

}  // extern "C"
