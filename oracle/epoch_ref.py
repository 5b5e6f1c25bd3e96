"""ORACLE (test infrastructure only) — restatement of the reference's per-batch train/test step.

Follows /root/reference/epoch_utils.py:
  train  :168-318   neg sample, per-block split (:209-213), n_id union (:215), sampler (:220),
                    CPU feature gather (:224), ones/zeros self-loop padding (:246-250),
                    graph (:254), forward (:262), BCE pos+neg (:295-296), insert (:300),
                    backward/step (:303-304), total_loss += loss*B (:310)
  test   :15-165    neg truncation to the batch minimum (:48-56), same assembly, forward with
                    neg_samples=K' (:99), MRR per batch (:108-113), insert (:157), mean (:163)
Negatives are injected (the reference's draw is unseeded, neg_sampler.py:11).
Also the timed CPU baseline ("port") of bench.py.
"""
from __future__ import annotations

import numpy as np
import torch

from .mrr_ref import mrr_batch
from .sampler_ref import RefLastNeighborLoader
from .tgnn_ref import RefGraph, RefTGNN


def _assemble(loader: RefLastNeighborLoader, feats, src, pos, neg, t, msg, b):
    k = int(b.max()) + 1
    srcs = [src[b == i] for i in range(k)]
    poss = [pos[b == i] for i in range(k)]
    negs = [neg[b == i] for i in range(k)]
    tx = [t[b == i] for i in range(k)]
    msgs = [msg[b == i] for i in range(k)]
    n_id = torch.cat([src, pos, neg.reshape(-1)]).unique()
    n_id, ei, e_id, bt = loader(n_id.numpy())
    bf = feats[torch.from_numpy(e_id)]
    M = n_id.shape[0]
    bf = torch.cat([bf, torch.ones(M, feats.shape[1])], dim=0)
    bt = torch.cat([torch.from_numpy(bt), torch.zeros(M)], dim=0)
    g = RefGraph(torch.from_numpy(ei[0]), torch.from_numpy(ei[1]), torch.from_numpy(n_id), self_loop=True)
    assoc = torch.from_numpy(loader._assoc)
    return g, bf, bt, (srcs, poss, negs, tx, msgs, assoc)


def train_batch(model: RefTGNN, opt, loader, feats, src, pos, neg, t, msg, b):
    """One iteration of epoch_utils.py:186-315. Returns (loss, pos_out, neg_out)."""
    opt.zero_grad()
    g, bf, bt, blocks = _assemble(loader, feats, src, pos, neg, t, msg, b)
    pos_out, neg_out = model(g, bf, bt, blocks)
    crit = torch.nn.BCEWithLogitsLoss()
    loss = crit(pos_out, torch.ones_like(pos_out))
    loss = loss + crit(neg_out, torch.zeros_like(neg_out))
    loader.insert(src.numpy(), pos.numpy(), t.numpy())
    loss.backward()
    opt.step()
    return loss.detach(), pos_out.detach(), neg_out.detach()


@torch.no_grad()
def eval_batch(model: RefTGNN, loader, feats, src, pos, neg2d, t, msg, b):
    """One iteration of epoch_utils.py:28-157 (after the negative truncation). Returns
    (mrr, pos_out[B], neg_out[B, K'])."""
    g, bf, bt, blocks = _assemble(loader, feats, src, pos, neg2d, t, msg, b)
    pos_out, neg_out = model(g, bf, bt, blocks, neg_samples=neg2d.shape[1])
    neg_out = neg_out.view(pos_out.shape[0], -1, 1)
    mrr = mrr_batch(pos_out.squeeze(-1).numpy(), neg_out.squeeze(-1).numpy())
    loader.insert(src.numpy(), pos.numpy(), t.numpy())
    return mrr, pos_out.squeeze(-1), neg_out.squeeze(-1)


def truncate_negatives(neg_rows) -> np.ndarray:
    """epoch_utils.py:48-56: every row cut to the batch's shortest negative list."""
    m = min(len(r) for r in neg_rows)
    return np.asarray([list(r)[:m] for r in neg_rows], dtype=np.int64)
