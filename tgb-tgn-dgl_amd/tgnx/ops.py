"""torch.ops.tgnx — libtgnx's C ABI registered as PyTorch operators (csrc/tgnx_torch.cpp).

    from tgnx import ops; ops.load()
    n_id, edge_index, e_id, t = torch.ops.tgnx.ring_sample(nbr, e_id, t, assoc, n_id)

Ops: ring_reset / ring_sample / ring_insert (LastNeighborLoader, neighbor_loader.py:26-109), neg_sample
(NegLinkSamplerDest, neg_sampler.py:8-23), block_ids (dependencyGraph.py:8-49, host tensors), tcsr_build /
tcsr_sample (TGL t-CSR, utils.py:73), gemm_f32 (MFMA fp32 GEMM), and the TGN modules' operators one call each
(csrc/tgnx_ops.hip): msg_agg_last / msg_agg_mean (LastAggregator / MeanAggregator, modules/msg_agg.py:15-26),
gru_update (TGNMemory's GRUCell / RNNCell, memory_module.py:70-78), predictor (LinkPredictor decoder.py:12-27;
EdgePredictor model_utils.py:165-195) and edge_attn_fwd / edge_attn_bwd (TransformerConv's attention,
emb_module.py:21-29; `edge_attention` below wraps the pair as an autograd function).  No CPU fallback: loading
needs the built library (make -C tgb-tgn-dgl_amd) and the device ops need a HIP device.
"""
from __future__ import annotations

import os

import torch

OPS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libtgnx_torch.so")
OPS = ("ring_reset", "ring_sample", "ring_insert", "neg_sample", "block_ids", "tcsr_build", "tcsr_sample", "gemm_f32",
       "msg_agg_last", "msg_agg_mean", "gru_update", "predictor", "edge_attn_fwd", "edge_attn_bwd",
       "sample_recent", "insert_recent", "reset")
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


class _EdgeAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, e, indptr, heads):
        out, alpha = load().edge_attn_fwd(q, k, v, e, indptr, heads)
        ctx.save_for_backward(q, k, v, e if e is not None else q.new_empty(0), indptr, alpha)
        ctx.heads, ctx.has_e = heads, e is not None
        ctx.mark_non_differentiable(alpha)
        return out, alpha

    @staticmethod
    def backward(ctx, dout, _dalpha):
        q, k, v, e, indptr, alpha = ctx.saved_tensors
        dq, dk, dv, de = load().edge_attn_bwd(dout.contiguous(), q, k, v, e if ctx.has_e else None, indptr, alpha,
                                              ctx.heads)
        return dq, dk, dv, (de if ctx.has_e else None), None, None


def edge_attention(q, k, v, e, indptr, heads):
    """TransformerConv's attention (PyG semantics, emb_module.py:21-29) with autograd: q [n_dst, H*C] per
    destination; k, v, e [E, H*C] per edge, destination i's edges the rows [indptr[i], indptr[i+1]) (e may be
    None).  Returns (out [n_dst, H*C], alpha [E, H]); gradients flow to q, k, v, e."""
    return _EdgeAttention.apply(q.contiguous(), k.contiguous(), v.contiguous(),
                                None if e is None else e.contiguous(), indptr, int(heads))
