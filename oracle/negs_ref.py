"""ORACLE (test infrastructure only) — restatement of `NegLinkSamplerDest.sample`.

Follows /root/reference/neg_sampler.py:8-23: draw `torch.randint(0, len(dst_nodes), (n,))`
from torch's global CPU generator, index the destination list, and recursively
redraw (same recipe, on the colliding subset only) wherever the draw equals the
positive.  Replaying torch's generator makes this bit-exact with the reference
(tests/golden/negs.npz).  The HIP sampler cannot share torch's CPU stream; it is
checked for the same distribution (uniform over destinations minus the positive).
"""
from __future__ import annotations

import torch


def sample(dst_nodes: torch.Tensor, pos_dst: torch.Tensor) -> torch.Tensor:
    cand = dst_nodes.tolist()
    draw = torch.randint(0, len(cand), (pos_dst.shape[0],))
    neg = torch.tensor([cand[i] for i in draw.tolist()], dtype=pos_dst.dtype)
    bad = (neg == pos_dst).nonzero(as_tuple=True)
    if bad[0].numel() > 0:
        neg[bad] = sample(dst_nodes, pos_dst[bad])
    return neg
