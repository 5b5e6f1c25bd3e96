"""train / test of the PyG TGN memory path (the canonical loop the reference's
pyg_epoch_utils.py:9-147 carries commented out, :106-137) on the fused HIP step (tgnx.tgn.TgnEngine).

  train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion)
      -> total_loss = Σ_batches loss·B (pyg_epoch_utils.py:138); prints "ap and auc: ..." (:139-147)
  test(model, feats, loader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion,
       evaluator, metric, split_mode) -> mean over batches of the batch MRR (epoch_utils.py:163)

Per train epoch: memory.reset_state + neighbor_loader.reset_state (pyg_epoch_utils.py:15-16), then the
bench's step (the parity-set step replayed from captured HIP graphs, TgnEngine.replay_resident); per
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
        # the per-event train-output log (tgnx_tgn_buffers.out_ev): every replayed step writes its batch's
        # outputs at their event rows, so the epoch's AP / AUC need no copy per step
        eng.out_ev = torch.zeros(eng.cfg.num_events, 2, dtype=torch.float32, device=eng.dev)
        eng.keep_grads = False    # the loop never reads the gradients (Adam fused: TGNX_TGN_NO_GRAD_STORE)
        eng._mode_train = None
        eng._bound = None
        m._tgnx_engine = eng
    return eng


def ap_auc_rows(pos: torch.Tensor, neg: torch.Tensor, chunk_elems: int = 1 << 26):
    """sklearn's average_precision_score / roc_auc_score of each row's labels [1]*P + [0]*N on the scores
    [pos | neg] (pyg_epoch_utils.py:139-143), for a [R, P] / [R, N] pair of score tensors, on their device.
    AUC = the Mann-Whitney statistic with ties counted 1/2 (roc_auc_score's trapezoids); AP = Σ over distinct
    thresholds of Δrecall x precision, i.e. the mean over positives of the precision at the end of their
    tie group (average_precision_score).  Returns float64 [R] tensors (ap, auc)."""
    R, Pn = pos.shape
    Nn = neg.shape[1]
    if R == 0:
        z = torch.zeros(0, dtype=torch.float64, device=pos.device)
        return z, z
    step = max(1, chunk_elems // max(1, Pn * Nn))
    aucs, aps = [], []
    for a in range(0, R, step):
        p, n = pos[a:a + step], neg[a:a + step]
        gt = (p[:, :, None] > n[:, None, :]).sum((1, 2)).double()
        eq = (p[:, :, None] == n[:, None, :]).sum((1, 2)).double()
        aucs.append((gt + 0.5 * eq) / (Pn * Nn))
        sc = torch.cat([p, n], 1)
        y = torch.cat([torch.ones_like(p), torch.zeros_like(n)], 1).double()
        order = torch.argsort(sc, dim=1, descending=True, stable=True)
        ss, yy = sc.gather(1, order), y.gather(1, order)
        tp = yy.cumsum(1)
        asc = (-ss).contiguous()                                   # ascending rows
        end = torch.searchsorted(asc, asc, right=True) - 1         # last position of each tie group
        prec = tp.gather(1, end) / (end + 1).double()
        aps.append((yy * prec).sum(1) / Pn)
    return torch.cat(aps), torch.cat(aucs)


def epoch_ap_auc(out_ev: torch.Tensor, lo: int, hi: int, B: int):
    """Mean over the epoch's batches of the batch AP and AUC (pyg_epoch_utils.py:139-145) from the per-event
    output log: y_pred = sigmoid of the model's sigmoid outputs, as the reference computes it."""
    sc = torch.sigmoid(out_ev[lo:hi])
    n = hi - lo
    full = n // B
    ap, auc = ap_auc_rows(sc[:full * B, 0].view(full, B), sc[:full * B, 1].view(full, B))
    if n > full * B:
        a2, u2 = ap_auc_rows(sc[full * B:, 0].view(1, -1), sc[full * B:, 1].view(1, -1))
        ap, auc = torch.cat([ap, a2]), torch.cat([auc, u2])
    return float(ap.mean()), float(auc.mean())


def train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion):
    """One train epoch as the benchmark runs it: the split bound resident, then the parity-set step replayed
    from its captured graphs batch after batch (TgnEngine.replay_resident; the first step of the epoch runs
    eagerly and prefetches the next), negatives drawn on the device, outputs logged per event."""
    eng = _engine(model, train_loader, neighbor_loader, optimizer, neg_dest_sampler)
    B = train_loader.batch_size
    key = (train_loader.lo, train_loader.hi, B)
    if eng._bound != key:
        eng.bind_resident(train_loader.lo, train_loader.hi, B, dropout=True)
        eng._bound = key
        eng._graphs = None
    eng.begin_epoch()                                     # pyg_epoch_utils.py:15-16 (+ the batch cursor)
    eng._mode_train = True
    loss0 = eng.loss_sum()
    if getattr(eng, "_graphs", None) is None:
        eng.capture_resident()
        eng.capture_group(8)                              # (world 1: 8 steps per graph launch)
    eng.replay_resident_n(len(train_loader))
    eng.finish()
    neighbor_loader.cur_e_id = train_loader.hi
    loss = eng.loss_sum() - loss0                         # (synchronises)
    eng.check()
    if train_loader.hi > train_loader.lo:
        ap, auc = epoch_ap_auc(eng.out_ev, train_loader.lo, train_loader.hi, B)
        print("ap and auc: ", ap, auc)
    return loss


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
