"""ctypes binding of libtgnx.so (the C ABI declared in include/tgnx.h).

The product path has no CPU fallback: if the library is missing or no HIP
device is visible, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TGNX_LIB") or os.path.join(_HERE, "libtgnx.so")

c_i32, c_i64, c_u64, c_sz, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
P = c_vp  # every device pointer crosses as void*

# name -> (restype, argtypes); must match include/tgnx.h
SIGNATURES = {
    "tgnx_version": (ctypes.c_int, []),
    "tgnx_last_error": (ctypes.c_char_p, []),
    "tgnx_ring_reset": (ctypes.c_int, [P, P, c_i64, c_i32, c_vp]),
    "tgnx_ring_sample_ws_bytes": (c_sz, [c_i64, c_i64]),
    "tgnx_ring_sample": (ctypes.c_int, [P, P, P, c_i64, c_i32, P, c_i64, P, P, P, P, P, c_i64, c_i64, P, P, c_sz,
                                        c_vp]),
    "tgnx_ring_insert_max_batch": (ctypes.c_int, []),
    "tgnx_ring_insert": (ctypes.c_int, [P, P, P, c_i64, c_i32, P, P, P, c_i64, c_i64, P, c_vp]),
    "tgnx_neg_sample": (ctypes.c_int, [P, c_i64, P, c_i64, c_u64, c_u64, P, c_vp]),
    "tgnx_block_ids_host": (ctypes.c_int, [P, P, c_i64, c_i64, P]),
    "tgnx_probe_enable": (ctypes.c_int, [c_i32]),
    "tgnx_probe_read": (ctypes.c_int, [P, P]),
    "tgnx_stamps_set": (ctypes.c_int, [P, ctypes.c_uint32]),
    "tgnx_stamps_count": (c_i64, []),
    "tgnx_tgnn_param_layout": (ctypes.c_int, [P, P]),
    "tgnx_tgnn_ws_bytes": (c_sz, [P]),
    "tgnx_tgnn_ws_misc_offset": (c_sz, [P]),
    "tgnx_tgn_param_layout": (ctypes.c_int, [P, P]),
    "tgnx_tgn_ws_bytes": (c_sz, [P]),
    "tgnx_tgn_store_words": (c_sz, [P]),
    "tgnx_tgn_reset_state": (ctypes.c_int, [P, P, c_vp]),
    "tgnx_tgn_plan_table_bytes": (c_sz, [P, c_i64, c_i64, c_i64]),
    "tgnx_tgn_plan_table": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, P, c_sz, c_vp]),
    "tgnx_tgn_plan_table_release": (ctypes.c_int, [P]),
    "tgnx_tgn_train_fwd_bwd": (ctypes.c_int, [P, P, c_i32, c_i32, c_vp]),
    "tgnx_tgn_train_update": (ctypes.c_int, [P, P, c_vp]),
    "tgnx_tgn_train_step": (ctypes.c_int, [P, P, c_i32, c_i32, c_vp]),
    "tgnx_tgn_train_step_resident": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_i32, c_vp]),
    "tgnx_tgn_train_step_pipelined": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_u64, c_i32, c_i32, c_vp]),
    "tgnx_tgn_train_step_pp": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_u64, c_i32, c_i32, c_i32, c_vp]),
    "tgnx_tgn_train_fwd_bwd_resident": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_i32, c_vp]),
    "tgnx_tgn_train_fwd_bwd_pipelined": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_i32, c_i32,
                                                         c_vp]),
    "tgnx_tgn_apply_rows_update": (ctypes.c_int, [P, P, P, c_i64, c_vp]),
    "tgnx_tgn_train_fwd_bwd_split": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_i32, c_i32, c_vp]),
    "tgnx_tgn_train_fwd_bwd_pp": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_i32, c_i32, c_i32,
                                                  c_i32, P, c_i64, c_vp]),
    "tgnx_tgn_scan_next": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_vp]),
    "tgnx_tgn_eval_step": (ctypes.c_int, [P, P, c_i32, c_vp]),
    "tgnx_tgn_flush": (ctypes.c_int, [P, P, P, ctypes.c_size_t, c_vp]),
    "tgnx_tgn_flush_scratch_bytes": (ctypes.c_size_t, [P]),
    "tgnx_tgn_apply_rows": (ctypes.c_int, [P, P, P, c_i64, c_vp]),
    "tgnx_tcsr_build_ws_bytes": (c_sz, [c_i64, c_i32]),
    "tgnx_tcsr_build": (ctypes.c_int, [P, P, P, c_i64, c_i64, c_i32, P, P, P, P, P, P, c_sz, c_vp]),
    "tgnx_tcsr_sample": (ctypes.c_int, [P, P, P, P, c_i64, c_i32, P, c_i64, c_i32, P, c_i64, P, P, P, P, P, c_vp]),
    "tgnx_gemm_f32_ws_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "tgnx_gemm_f32": (ctypes.c_int, [c_i64, c_i64, c_i64, P, c_i64, c_i32, P, c_i64, c_i32, P, c_i64, P, c_i32, P, c_sz,
                                     c_vp]),
    # per-operator entry points (tgnx_ops.hip)
    "tgnx_msg_agg_ws_bytes": (c_sz, [c_i64, c_i64]),
    "tgnx_msg_agg": (ctypes.c_int, [c_i32, P, c_i64, c_i64, P, P, c_i32, c_i64, P, P, P, P, c_sz, c_vp]),
    "tgnx_memory_cell_ws_bytes": (c_sz, [c_i64, c_i64, c_i64]),
    "tgnx_memory_cell": (ctypes.c_int, [c_i32, c_i64, c_i64, c_i64, P, P, P, P, P, P, P, P, c_sz, c_vp]),
    "tgnx_link_predictor_ws_bytes": (c_sz, [c_i64, c_i64, c_i64, c_i64]),
    "tgnx_link_predictor": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i64, P, P, P, P, P, P, P, P, c_i32, P, P, c_sz,
                                           c_vp]),
    "tgnx_edge_attn_fwd": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32, P, P, P, P, P, P, P, c_vp]),
    "tgnx_edge_attn_bwd": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32, P, P, P, P, P, P, P, P, P, P, P, c_vp]),
    "tgnx_tgnn_advance": (ctypes.c_int, [P, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64,
                                         c_i32, c_vp]),
    "tgnx_tgnn_train_fwd_bwd": (ctypes.c_int, [P, P, c_i32, c_i32, c_vp]),
    "tgnx_tgnn_train_fwd_bwd_resident": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_i32, c_i32, c_u64, c_i32, c_vp]),
    "tgnx_tgnn_train_step_resident": (ctypes.c_int, [P, P, c_i64, c_i64, c_i64, c_u64, c_i32, c_vp]),
    "tgnx_tgnn_apply_pending": (ctypes.c_int, [P, P, c_vp]),
    "tgnx_tgnn_train_update": (ctypes.c_int, [P, P, c_vp]),
    "tgnx_tgnn_eval_step": (ctypes.c_int, [P, P, c_i32, c_i32, c_vp]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"tgnx: {LIB_PATH} is missing — build it with `make -C tgb-tgn-dgl_amd` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("TGNX_LIB") and not hasattr(L, name):
                continue    # (an older library selected for a same-box A/B: entry points it predates stay unbound)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().tgnx_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def ptr(t: torch.Tensor | None):
    return c_vp(0 if t is None else t.data_ptr())


def stream(device: torch.device | None = None):
    return c_vp(torch.cuda.current_stream(device).cuda_stream)


def require_device(device) -> torch.device:
    dev = torch.device(device) if device is not None else torch.device("cuda")
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("tgnx runs only on a HIP device (MI355X); got device=%r, "
                           "torch.cuda.is_available()=%s" % (device, torch.cuda.is_available()))
    lib()
    return dev
