"""Time tgnx_gemm_f32 against torch.matmul (hipBLASLt) at the TGN step's GEMM shapes."""
import ctypes
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tgb-tgn-dgl_amd"))
import torch
from tgnx import _lib

dev = torch.device("cuda")
for (M, N, K, ta, tb) in [(413, 400, 572, 0, 1), (1826, 100, 272, 0, 1), (100, 272, 1826, 1, 0), (400, 101, 413, 1, 0),
                          (413, 100, 400, 0, 0), (400, 573, 413, 1, 0), (6600, 400, 572, 0, 1)]:
    A = torch.randn((K, M) if ta else (M, K), device=dev)
    B = torch.randn((N, K) if tb else (K, N), device=dev)
    C = torch.zeros(M, N, device=dev)
    nb = _lib.lib().tgnx_gemm_f32_ws_bytes(M, N, K)
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    st = _lib.stream()

    def run():
        _lib.call("tgnx_gemm_f32", M, N, K, _lib.ptr(A), A.shape[1], ta, _lib.ptr(B), B.shape[1], tb, _lib.ptr(C), N,
                  None, 0, _lib.ptr(ws), ctypes.c_size_t(nb), st)
    opA = A.t() if ta else A
    opB = B.t() if tb else B
    for f, name in ((run, "tgnx"), (lambda: torch.matmul(opA, opB), "torch")):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        print(f"M={M} N={N} K={K} ta={ta} tb={tb} {name}: {us:.1f} us  {2*M*N*K/us/1e6:.2f} TFLOP/s")
