"""The split-K MFMA fp32 GEMM behind the TGN memory path (include/tgnx.h tgnx_gemm_f32) against a
plain torch fp32 matmul: all four transpose modes, split-K (K > 64), ragged edges, bias,
accumulate, determinism."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _gemm(A, B, ta, tb, M, N, K, bias=None, C=None, acc=False):
    from tgnx import _lib
    dev = A.device
    if C is None:
        C = torch.zeros(M, N, device=dev)
    nb = _lib.lib().tgnx_gemm_f32_ws_bytes(M, N, K)
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    lda, ldb = A.shape[1], B.shape[1]
    _lib.call("tgnx_gemm_f32", M, N, K, _lib.ptr(A), lda, int(ta), _lib.ptr(B), ldb, int(tb), _lib.ptr(C), N,
              _lib.ptr(bias) if bias is not None else None, int(acc), _lib.ptr(ws), ctypes.c_size_t(nb),
              _lib.stream())
    return C


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (17, 33, 5), (64, 64, 64), (413, 400, 572), (100, 272, 1710),
                                   (3, 100, 413)])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 1), (1, 0)])
def test_gemm_matches_torch(M, N, K, ta, tb):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    dev = torch.device("cuda")
    A = torch.randn((K, M) if ta else (M, K), generator=g).to(dev)
    B = torch.randn((N, K) if tb else (K, N), generator=g).to(dev)
    bias = torch.randn(N, generator=g).to(dev)
    opA = A.t() if ta else A
    opB = B.t() if tb else B
    ref = (opA.double() @ opB.double() + bias.double()).float()
    out = _gemm(A, B, ta, tb, M, N, K, bias=bias)
    torch.cuda.synchronize()
    tol = 1e-5 * (K ** 0.5) + 1e-6
    assert torch.allclose(out, ref, rtol=tol, atol=tol * 4), (out - ref).abs().max()
    out2 = _gemm(A, B, ta, tb, M, N, K, bias=bias)
    assert torch.equal(out, out2)           # fixed-order split-K reduction


def test_gemm_accumulate():
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(1)
    A, B = torch.randn(70, 130, generator=g).to(dev), torch.randn(90, 130, generator=g).to(dev)
    C0 = torch.randn(70, 90, generator=g).to(dev)
    out = _gemm(A, B, 0, 1, 70, 90, 130, C=C0.clone(), acc=True)
    ref = C0 + A @ B.t()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-4)
