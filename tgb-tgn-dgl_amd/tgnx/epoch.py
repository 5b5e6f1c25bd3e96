"""Drop-in `train` / `test` (epoch_utils.py:15-318) on the fused HIP step.

Same signatures and return values as the reference:
  train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion)
      -> total_loss = Σ_batches loss·B   (epoch_utils.py:310,318); prints "ap and auc: ..."
  test(model, feats, loader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion,
       evaluator, metric, split_mode) -> mean over batches of the batch MRR (epoch_utils.py:163)
Reference behaviour kept: the ring is reset at the start of every train epoch (:175) but
time_assoc is not; test() switches the model to eval and nothing switches it back, so
dropout (0.6) is active in the first epoch only (:20, :170-172); negatives are truncated
to the batch's shortest list (:48-56); the eval predictor pairs negative row r with source
r mod B (model_utils.py:192).

A {'memory', 'gnn', 'link_pred'} model (pyg_model_utils.getModel, the import swap at pyg-mem-tgn.py:23-25)
is handed to the PyG TGN loop (tgnx/tgn_epoch.py), so the reference script keeps its epoch_utils import.

With a tgnx SplitLoader the whole split is resident in HBM and each batch is a few C-ABI
calls with no host synchronisation; any other iterable of batch dicts is copied per batch.
"""
from __future__ import annotations

import numpy as np
import torch

from .data import SplitLoader
from .engine import TgnnEngine


def _engine(model, feats, neighbor_loader, optimizer, neg_dest_sampler=None, max_neg=1):
    gnn = model["gnn"] if isinstance(model, dict) else model
    eng = getattr(gnn, "_tgnx_engine", None)
    dst_nodes = getattr(neg_dest_sampler, "dst_nodes", None)
    if eng is None or eng.loader is not neighbor_loader or eng.cfg.max_neg < max_neg:
        if eng is not None and max_neg < eng.cfg.max_neg:
            max_neg = eng.cfg.max_neg
        if eng is not None and dst_nodes is None:
            dst_nodes = eng.dst_nodes
        old = eng
        if dst_nodes is not None and not torch.is_tensor(dst_nodes):
            dst_nodes = torch.as_tensor(dst_nodes, dtype=torch.long)
        eng = TgnnEngine(gnn, neighbor_loader, torch.as_tensor(feats), optimizer, dst_nodes=dst_nodes,
                         max_neg=max_neg, seed=getattr(neg_dest_sampler, "seed", 0))
        if old is not None:          # keep the step counters (Adam t, generation, loss) across re-binds
            eng.ctl.copy_(old.ctl)
        gnn._tgnx_engine = eng
    elif dst_nodes is not None and eng.dst_nodes is None:
        eng.dst_nodes = dst_nodes
    return gnn, eng


def _ap_auc(pos: np.ndarray, neg: np.ndarray):
    from sklearn.metrics import average_precision_score, roc_auc_score
    y = np.concatenate([np.ones_like(pos), np.zeros_like(neg)])
    p = 1.0 / (1.0 + np.exp(-np.concatenate([pos, neg])))
    return average_precision_score(y, p), roc_auc_score(y, p)


def _is_tgn(model) -> bool:
    """A {'memory', 'gnn', 'link_pred'} dict: pyg_model_utils.getModel (the import swap at
    pyg-mem-tgn.py:23-25), trained by the PyG TGN loop (tgnx/tgn_epoch.py)."""
    return isinstance(model, dict) and "memory" in model and "link_pred" in model


def train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer, criterion):
    if _is_tgn(model):
        from . import tgn_epoch
        return tgn_epoch.train(model, feats, train_loader, neighbor_loader, neg_dest_sampler, assoc, device,
                               optimizer, criterion)
    gnn, eng = _engine(model, feats, neighbor_loader, optimizer, neg_dest_sampler)
    neighbor_loader.reset_state()                       # epoch_utils.py:175
    eng.reset_loss()
    if isinstance(train_loader, SplitLoader):
        # the split resident in HBM, the step replayed from a captured HIP graph batch after batch (what the
        # benchmark times); every step writes its logits at their event rows of the per-event log
        ev = train_loader.resident(eng.dev)
        n = train_loader.data.num_events
        neg_buf = getattr(eng, "_train_neg_buf", None)
        if neg_buf is None or neg_buf.numel() < n:
            neg_buf = eng._train_neg_buf = torch.zeros(n, dtype=torch.long, device=eng.dev)
        if eng.out_ev is None or eng.out_ev.shape[0] < n:
            eng.out_ev = torch.zeros(n, 2, dtype=torch.float32, device=eng.dev)
        B = train_loader.batch_size
        # the captured graph bakes in every pointer of the step's buffer block (events, negatives, output log,
        # destination set, parameters, optimizer state, workspace, ring): key it on all of them
        bufs = eng._buffers(ev["src"], ev["dst"], ev["t"], ev["blk"], ev["msg"], neg_buf)
        key = (train_loader.lo, train_loader.hi, B, gnn.training, bytes(bufs))
        if getattr(eng, "_bound", None) != key:   # (gnn.training: dropout of the first epoch only, :170-172)
            eng.bind_resident(ev["src"], ev["dst"], ev["t"], ev["blk"], ev["msg"], neg_buf, train_loader.lo,
                              train_loader.hi, B)
            eng.capture_resident(1)
            eng.capture_group(8)                         # (world 1: 8 steps per graph launch)
            eng._bound = key
        eng.ctl[10] = 0
        eng.replay_resident_n(len(train_loader))
        eng.finish()                                     # the last step's update (deferred by the resident step)
        neighbor_loader.cur_e_id = train_loader.hi       # e_ids are global event rows (val continues)
        torch.cuda.synchronize(eng.dev)
        eng.check()
        if train_loader.hi > train_loader.lo:           # epoch_utils.py:312-317 (display only)
            from .tgn_epoch import epoch_ap_auc
            ap, auc = epoch_ap_auc(eng.out_ev, train_loader.lo, train_loader.hi, B)
            print("ap and auc: ", ap, auc)
        return eng.loss_sum()
    logits = []
    for batch in train_loader:
        pos, neg, _ = eng.train_batch(batch["src"], batch["dst"], batch["t"], batch["msg"], batch["b"])
        logits.append(torch.stack([pos.clone(), neg.clone()]))
    torch.cuda.synchronize(eng.dev)
    eng.check()
    aps, aucs = [], []
    for lg in logits:                                     # epoch_utils.py:312-317 (display only)
        lg = lg.cpu().numpy()
        ap, auc = _ap_auc(lg[0], lg[1])
        aps.append(ap)
        aucs.append(auc)
    if aps:
        print("ap and auc: ", float(np.mean(aps)), float(np.mean(aucs)))
    return eng.loss_sum()


@torch.no_grad()
def test(model, feats, loader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion, evaluator,
         metric, split_mode):
    if _is_tgn(model):
        from . import tgn_epoch
        return tgn_epoch.test(model, feats, loader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion,
                              evaluator, metric, split_mode)
    gnn = model["gnn"] if isinstance(model, dict) else model
    gnn.eval()                                           # epoch_utils.py:20 (never undone: reference quirk)
    perf = []
    if isinstance(loader, SplitLoader) and loader.negatives is not None:
        negs = loader.negatives
        kn = int(negs.shape[1])
        gnn, eng = _engine(model, feats, neighbor_loader, optimizer, max_neg=kn)
        ev = loader.resident(eng.dev)
        neg_dev = ev["neg"]
        for s in range(loader.lo, loader.hi, loader.batch_size):
            e = min(loader.hi, s + loader.batch_size)
            pos, neg, mrr = eng.eval_batch(ev["src"][s:e], ev["dst"][s:e], ev["t"][s:e], ev["msg"][s:e],
                                           ev["blk"][s:e], neg_dev[s - loader.lo:e - loader.lo])
            perf.append(mrr.clone())
    else:
        gnn, eng = _engine(model, feats, neighbor_loader, optimizer)
        for batch in loader:
            rows = neg_sampler.query_batch(batch["src"], batch["dst"], batch["t"], split_mode=split_mode)
            m = min(len(r) for r in rows)                 # epoch_utils.py:48-56
            neg2d = torch.tensor([list(r)[:m] for r in rows], dtype=torch.long)
            if m > eng.cfg.max_neg:
                gnn, eng = _engine(model, feats, neighbor_loader, optimizer, max_neg=m)
            pos, neg, mrr = eng.eval_batch(batch["src"], batch["dst"], batch["t"], batch["msg"], batch["b"], neg2d)
            perf.append(mrr.clone())
    torch.cuda.synchronize(eng.dev)
    eng.check()
    return float(torch.stack(perf).mean()) if perf else float("nan")
