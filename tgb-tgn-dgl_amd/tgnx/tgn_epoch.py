"""train / test of the PyG TGN memory path (the canonical loop the reference's
pyg_epoch_utils.py:9-147 carries commented out, :106-137) on the fused HIP step (tgnx.tgn.TgnEngine).

  train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion)
      -> total_loss = Σ_batches loss·B (pyg_epoch_utils.py:138); prints "ap and auc: ..." (:139-147)
  test(model, feats, loader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion,
       evaluator, metric, split_mode) -> mean over batches of the batch MRR (epoch_utils.py:163)

Per train epoch: memory.reset_state + neighbor_loader.reset_state (pyg_epoch_utils.py:15-16); per
batch: negatives from the destination set (NegLinkSamplerDest distribution, drawn on the device),
memory(n_id) with the GRU update of every sampled node, TransformerConv embedding, LinkPredictor,
BCE-with-logits on its sigmoid outputs (as the reference feeds it), update_state, ring insert,
backward, Adam.  test(): the first call after training switches the memory to eval
(TGNMemory.train(False): every node's memory updated from its stored messages, stores cleared,
memory_module.py:209-215); each batch scores [pos, negatives] with the batch-start state, then
updates the stores, the memory and the ring in eval order.

Reached through pyg_epoch_utils (shim) and through epoch_utils.train / test, which dispatch here for a
{'memory', 'gnn', 'link_pred'} model: the reference script runs with only its model import swapped
(pyg-mem-tgn.py:19 keeps `from epoch_utils import train, test`).

The loaders must be tgnx SplitLoaders (tgnx.data; what utils.getDataWithDependecyBlock returns):
the event table is bound resident in HBM once and batches address it by global row (e_id)."""
from __future__ import annotations

import numpy as np
import torch

from .data import SplitLoader
from .tgn import TgnEngine


def _owner(model):
    return model["model"] if isinstance(model, dict) else model


def _engine(model, train_loader, neighbor_loader, optimizer, neg_dest_sampler=None):
    m = _owner(model)
    eng = getattr(m, "_tgnx_engine", None)
    if eng is None or eng.loader is not neighbor_loader:
        if not isinstance(train_loader, SplitLoader):
            raise TypeError("tgnx pyg_epoch_utils needs tgnx.data.SplitLoader batches (the event table is "
                            "bound resident; see utils.getDataWithDependecyBlock)")
        d = train_loader.data
        dst_nodes = getattr(neg_dest_sampler, "dst_nodes", None)
        if dst_nodes is None:
            dst_nodes = torch.unique(torch.as_tensor(d.dst))
        eng = TgnEngine(m, neighbor_loader, dict(src=d.src, dst=d.dst, t=d.t.float(), msg=d.msg.float()),
                        optimizer, dst_nodes=torch.as_tensor(dst_nodes), seed=getattr(neg_dest_sampler, "seed", 0))
        eng._mode_train = None
        m._tgnx_engine = eng
    return eng


def _ap_auc(pos: np.ndarray, neg: np.ndarray):
    from sklearn.metrics import average_precision_score, roc_auc_score
    y = np.concatenate([np.ones_like(pos), np.zeros_like(neg)])
    p = np.concatenate([pos, neg])     # the sigmoid outputs (pyg_epoch_utils.py:141 applies one more)
    return average_precision_score(y, p), roc_auc_score(y, p)


def train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion):
    eng = _engine(model, train_loader, neighbor_loader, optimizer, neg_dest_sampler)
    eng.reset_state()                                     # pyg_epoch_utils.py:15-16
    eng._mode_train = True
    loss0 = eng.loss_sum()
    B = train_loader.batch_size
    outs = []
    for s in range(train_loader.lo, train_loader.hi, B):
        n = min(train_loader.hi, s + B) - s
        pos, neg = eng.train_batch(s, n)
        outs.append(torch.stack([pos.clone(), neg.clone()]))
    neighbor_loader.cur_e_id = train_loader.hi
    torch.cuda.synchronize(eng.dev)
    eng.check()
    aps, aucs = [], []
    for o in outs:
        o = o.cpu().numpy()
        ap, auc = _ap_auc(o[0], o[1])
        aps.append(ap)
        aucs.append(auc)
    if aps:
        print("ap and auc: ", float(np.mean(aps)), float(np.mean(aucs)))
    return eng.loss_sum() - loss0


@torch.no_grad()
def test(model, feats, loader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion, evaluator,
         metric, split_mode):
    eng = _engine(model, loader, neighbor_loader, optimizer)
    if eng._mode_train:                                   # TGNMemory.train(False) (memory_module.py:209-215)
        eng.flush()
        eng._mode_train = False
    perf = []
    B = loader.batch_size
    negs_all = loader.negatives
    for s in range(loader.lo, loader.hi, B):
        e = min(loader.hi, s + B)
        if negs_all is not None:
            negs = negs_all[s - loader.lo:e - loader.lo]
        else:
            d = loader.data
            rows = neg_sampler.query_batch(d.src[s:e], d.dst[s:e], d.t[s:e], split_mode=split_mode)
            m = min(len(r) for r in rows)                 # epoch_utils.py:48-56
            negs = torch.tensor([list(r)[:m] for r in rows], dtype=torch.long)
        _, _, rr = eng.eval_batch(s, e - s, negs)
        perf.append(rr.clone().mean())
    neighbor_loader.cur_e_id = loader.hi
    torch.cuda.synchronize(eng.dev)
    eng.check()
    return float(torch.stack(perf).mean()) if perf else float("nan")
