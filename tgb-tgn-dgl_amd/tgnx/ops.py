"""torch.ops.tgnx — libtgnx's C ABI registered as PyTorch operators (csrc/tgnx_torch.cpp).

    from tgnx import ops; ops.load()
    n_id, edge_index, e_id, t = torch.ops.tgnx.ring_sample(nbr, e_id, t, assoc, n_id)

Ops: ring_reset / ring_sample / ring_insert (LastNeighborLoader, neighbor_loader.py:26-109), neg_sample
(NegLinkSamplerDest, neg_sampler.py:8-23), block_ids (dependencyGraph.py:8-49, host tensors), tcsr_build /
tcsr_sample (TGL t-CSR, utils.py:73), gemm_f32 (MFMA fp32 GEMM).  No CPU fallback: loading needs the built
library (make -C tgb-tgn-dgl_amd) and the device ops need a HIP device.
"""
from __future__ import annotations

import os

import torch

OPS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtgnx_torch.so")
OPS = ("ring_reset", "ring_sample", "ring_insert", "neg_sample", "block_ids", "tcsr_build", "tcsr_sample", "gemm_f32")
_loaded = False


def load():
    """Register torch.ops.tgnx.* (idempotent); returns the op namespace."""
    global _loaded
    if not _loaded:
        if not os.path.exists(OPS_PATH):
            raise RuntimeError(f"tgnx: {OPS_PATH} is missing — build it with `make -C tgb-tgn-dgl_amd`")
        torch.ops.load_library(OPS_PATH)
        _loaded = True
    return torch.ops.tgnx
