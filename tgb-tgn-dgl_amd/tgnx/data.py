"""Data + config surface of the reference (utils.py:17-67, temporal_dataset.py, dependencyGraph.py).

`getDataWithDependecyBlock(name, train_param)` returns the same 7-tuple as the
reference (utils.py:25,67): (data, train_dl, val_dl, test_dl, neg_sampler,
evaluator, metric).  TGB datasets cannot be downloaded here, so `name` is either
  * a TGB dataset name (tgbl-wiki / -review / -coin / -comment): the dataset on disk under
    $TGNX_TGB_ROOT (default "datasets", as utils.py:29) in py-tgb's raw layout (tgnx.tgb_io), else a
    synthetic stream with that dataset's published shape (tgnx.synth; TGNX_SYNTH_EVENTS scales it down), or
  * a path to an .npz holding src, dst, t, msg (+ optional val_neg / test_neg).
Loaders iterate host batches exactly like the reference's DataLoader (dicts of
src/dst/t/msg/b/idx, t cast to float32 — temporal_dataset.py:34-57) and also carry
the whole split resident in HBM so tgnx.epoch.train/test run without per-batch copies.
Dependency-block ids (dependencyGraph.py:8-49) come from the native single-pass
`tgnx_block_ids_host` instead of the per-edge Python loop.
Reference quirk kept: the val loader gets the blocks computed on the test split and
vice versa (utils.py:55-61, "test_blocks = dab(val_dl)").
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import yaml

from . import _lib
from .synth import SHAPES, eval_negatives, make_stream
from .tgb_io import load_tgb, uniform_negatives


# sections of the configs parse_config returned, by the identity of their gnn section: the reference's
# script passes only gnn_param to getModel (pyg-mem-tgn.py:36,49), so pyg_model_utils.getModel finds the
# memory / sampling / train sections of the same file through it (memory.mail_combine, memory_update)


class GnnSection(dict):
    """The `gnn` section parse_config returns: a plain dict that also carries its file's sibling sections
    (sampling, memory, train), so that getModel(..., gnn_param=gnn) as pyg-mem-tgn.py:49 calls it can honour
    mail_combine / memory_update / neighbor / batch_size.  Explicit getModel keywords override them; a copy
    made with dict(gnn) carries only the gnn keys."""
    __slots__ = ("sections",)


def parse_config(f):
    """utils.py:17-23."""
    with open(f, "r") as fh:
        conf = yaml.safe_load(fh)
    gnn = GnnSection(conf["gnn"][0])
    out = conf["sampling"][0], conf["memory"][0], gnn, conf["train"][0]
    gnn.sections = out
    return out


def config_of(gnn_param):
    """(sampling, memory, gnn, train) of the parse_config call that returned this gnn section, or None."""
    got = getattr(gnn_param, "sections", None)
    return got if got is not None and got[2] is gnn_param else None


def block_ids(src: np.ndarray, dst: np.ndarray, batch: int) -> np.ndarray:
    """dependecyAwareBatch(flat=True) (dependencyGraph.py:33-49) in native code."""
    src = np.ascontiguousarray(src, dtype=np.int64)
    dst = np.ascontiguousarray(dst, dtype=np.int64)
    out = np.empty_like(src)
    _lib.call("tgnx_block_ids_host", src.ctypes.data, dst.ctypes.data, src.shape[0], int(batch), out.ctypes.data)
    return out


def get_block(tss, src_b, dst_b):
    """dependencyGraph.py:8-28 (one batch)."""
    return block_ids(np.asarray(src_b), np.asarray(dst_b), max(1, len(src_b))).tolist()


def dependecyAwareBatch(loader, flat=True):
    """dependencyGraph.py:33-49."""
    out = []
    for b in loader:
        blk = get_block(b["t"], b["src"], b["dst"])
        if flat:
            out.extend(blk)
        else:
            out.append(blk)
    return out


class TemporalGraphDataset(torch.utils.data.Dataset):
    """temporal_dataset.py:4-57 (items are dicts; t is cast to float32)."""

    def __init__(self, src, dst, t, msg, batch=None):
        self.src, self.dst, self.t, self.msg, self.batch = src, dst, t, msg, batch

    def __len__(self):
        return len(self.src)

    def __getitem__(self, idx):
        item = {"src": self.src[idx], "dst": self.dst[idx], "t": self.t[idx].float(), "msg": self.msg[idx]}
        if self.batch is not None:
            item["b"] = self.batch[idx]
        item["idx"] = idx
        return item


@dataclass
class TemporalData:
    """The fields of PyG TemporalData the reference reads (utils.py:34-40, pyg-mem-tgn.py:39-49)."""
    src: torch.Tensor
    dst: torch.Tensor
    t: torch.Tensor
    msg: torch.Tensor

    @property
    def num_nodes(self) -> int:
        return int(max(int(self.src.max()), int(self.dst.max())) + 1)

    @property
    def num_events(self) -> int:
        return int(self.src.shape[0])


class SplitLoader:
    """Batches of one chronological split, host-iterable like the reference's DataLoader and
    device-resident for the fused path (global event index = row of `data`)."""

    def __init__(self, data: TemporalData, lo: int, hi: int, batch_size: int, blocks: np.ndarray,
                 negatives: np.ndarray | None = None):
        self.data, self.lo, self.hi, self.batch_size = data, int(lo), int(hi), int(batch_size)
        self.blocks = torch.from_numpy(np.ascontiguousarray(blocks, dtype=np.int64))
        self.negatives = None if negatives is None else torch.from_numpy(np.ascontiguousarray(negatives))
        self._dev = {}

    def __len__(self):
        return math.ceil((self.hi - self.lo) / self.batch_size)

    def __iter__(self):
        d = self.data
        for s in range(self.lo, self.hi, self.batch_size):
            e = min(self.hi, s + self.batch_size)
            yield {"src": d.src[s:e], "dst": d.dst[s:e], "t": d.t[s:e].float(), "msg": d.msg[s:e],
                   "b": self.blocks[s - self.lo:e - self.lo], "idx": torch.arange(s - self.lo, e - self.lo)}

    def resident(self, device) -> dict:
        """Whole-stream event arrays (global index) on `device`; blocks / negatives padded to it."""
        key = str(device)
        if key not in self._dev:
            d = self.data
            n = d.num_events
            blk = torch.zeros(n, dtype=torch.long)
            blk[self.lo:self.hi] = self.blocks
            out = {"src": d.src.to(device), "dst": d.dst.to(device), "t": d.t.float().to(device),
                   "blk": blk.to(device), "msg": d.msg.float().contiguous().to(device)}
            if self.negatives is not None:
                out["neg"] = self.negatives.to(device).contiguous()
            self._dev[key] = out
        return self._dev[key]


class NegativeSampler:
    """Stands in for TGB's precomputed negative sampler (epoch_utils.py:43): query_batch returns,
    per positive, its list of negatives.  Batches of a split are served in order (a cursor per
    split), as the reference's loop consumes them; reset() rewinds."""

    def __init__(self, splits: dict):
        self.splits = splits   # name -> (first global event index, negatives [n, K'])
        self._cursor = {}

    def query_batch(self, src, pos_dst, t, split_mode="val"):
        _, neg = self.splits[split_mode]
        cur = self._cursor.get(split_mode, 0)
        n = len(src)
        self._cursor[split_mode] = cur + n
        return [list(r) for r in neg[cur:cur + n]]

    def reset(self, split_mode=None):
        if split_mode is None:
            self._cursor = {}
        else:
            self._cursor.pop(split_mode, None)


class Evaluator:
    """TGB link-prediction evaluator (MRR): rank = 0.5 (#neg > pos + #neg >= pos) + 1."""

    def __init__(self, name=None):
        self.name = name

    def eval(self, input_dict):
        pos = np.asarray(input_dict["y_pred_pos"], dtype=np.float64).reshape(-1, 1)
        neg = np.asarray(input_dict["y_pred_neg"], dtype=np.float64)
        rank = 0.5 * ((neg > pos).sum(1) + (neg >= pos).sum(1)) + 1.0
        return {"mrr": float((1.0 / rank).mean())}


def _load(name: str):
    if os.path.exists(name) and name.endswith(".npz"):
        z = np.load(name, allow_pickle=False)
        src, dst, t, msg = z["src"], z["dst"], z["t"], z["msg"]
        E = src.shape[0]
        tr, va = int(round(0.70 * E)), int(round(0.85 * E))
        negs = {k: z[k] for k in ("val_neg", "test_neg") if k in z.files}
        return src, dst, t, msg, tr, va, negs, None
    if name not in SHAPES:
        raise ValueError(f"unknown dataset {name!r}: give a TGB name {sorted(SHAPES)} or an .npz path")
    # a TGB dataset on disk (utils.py:29 reads datasets/<name>): raw edge list or the tgnx cache
    disk = load_tgb(name, root=os.environ.get("TGNX_TGB_ROOT", "datasets"),
                    allow_pickle=os.environ.get("TGNX_TGB_ALLOW_PICKLE") == "1")
    if disk is not None:
        src, dst, t, msg, tr, va, negs = disk
        kneg = int(os.environ.get("TGNX_EVAL_NEGS", str(SHAPES[name].num_neg_eval)))
        if "val_neg" not in negs:
            negs["val_neg"] = uniform_negatives(dst, tr, va, kneg, seed=1)
        if "test_neg" not in negs:
            negs["test_neg"] = uniform_negatives(dst, va, len(t), kneg, seed=2)
        return src, dst, t, msg, tr, va, negs, None
    ev = os.environ.get("TGNX_SYNTH_EVENTS")
    s = make_stream(SHAPES[name], seed=int(os.environ.get("TGNX_SYNTH_SEED", "0")),
                    num_events=int(ev) if ev else None)
    kneg = int(os.environ.get("TGNX_EVAL_NEGS", str(s.shape.num_neg_eval)))
    negs = {"val_neg": eval_negatives(s, "val", kneg), "test_neg": eval_negatives(s, "test", kneg)}
    return s.src, s.dst, s.t, s.msg, s.train_end, s.val_end, negs, s


def getDataWithDependecyBlock(DATA, train_param, csv=False, load_neg_sampler=True):
    """utils.py:25-67."""
    src, dst, t, msg, tr, va, negs, _ = _load(DATA)
    data = TemporalData(torch.from_numpy(np.asarray(src, dtype=np.int64)),
                        torch.from_numpy(np.asarray(dst, dtype=np.int64)),
                        torch.from_numpy(np.asarray(t, dtype=np.float64)),
                        torch.from_numpy(np.asarray(msg, dtype=np.float32)))
    E = data.num_events
    bs = int(train_param["batch_size"])
    b_train = block_ids(src[:tr], dst[:tr], bs)
    b_val = block_ids(src[tr:va], dst[tr:va], bs)
    b_test = block_ids(src[va:], dst[va:], bs)
    # utils.py:55-61: val batches carry the blocks computed on the test split and vice versa
    n_val, n_test = va - tr, E - va
    val_blocks = _fit(b_test, n_val)
    test_blocks = _fit(b_val, n_test)
    train_dl = SplitLoader(data, 0, tr, bs, b_train)
    val_dl = SplitLoader(data, tr, va, bs, val_blocks, negs.get("val_neg"))
    test_dl = SplitLoader(data, va, E, bs, test_blocks, negs.get("test_neg"))
    neg_sampler = evaluator = None
    if load_neg_sampler:
        neg_sampler = NegativeSampler({"val": (tr, negs.get("val_neg")), "test": (va, negs.get("test_neg"))})
        evaluator = Evaluator(DATA)
    return data, train_dl, val_dl, test_dl, neg_sampler, evaluator, "mrr"


def _fit(blocks: np.ndarray, n: int) -> np.ndarray:
    """The swapped block lists have the other split's length; the reference's Dataset indexes
    them positionally (temporal_dataset.py:54), so keep the first n (pad with block 0)."""
    out = np.zeros(n, dtype=np.int64)
    m = min(n, blocks.shape[0])
    out[:m] = blocks[:m]
    return out
