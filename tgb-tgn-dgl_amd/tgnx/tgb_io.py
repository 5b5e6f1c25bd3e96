"""TGB on-disk formats for the reference's data seam (utils.py:25-67, which reads them through
py-tgb's `PyGLinkPropPredDataset(name, root="datasets")`, absent here).

py-tgb is not installed and nothing can be downloaded, so the layouts below restate py-tgb's published
conventions (PARITY UNPINNED: no TGB file or py-tgb output exists in this container to check against):

* dataset directory: `<root>/<name with '-' -> '_'>/`, e.g. `datasets/tgbl_wiki/`;
* raw edge list `<name>_edgelist_v2.csv` (or `<name>_edgelist.csv`):
    - tgbl-wiki (JODIE layout): header line, then `user, item, timestamp, state_label, f_1 .. f_172`;
      item ids are shifted past the users (dst = item + max(user) + 1), msg = the feature columns;
    - every other tgbl dataset: header line, then `timestamp, source, destination[, w_1 ..]` with
      string or integer node keys, relabelled to 0.. in order of first appearance over (source,
      destination) of each event; msg = the remaining numeric columns (a ones column when absent);
* chronological split (py-tgb `generate_splits`): val_time, test_time = the 0.70 / 0.85 quantiles of
  the timestamps; train = t <= val_time, val = val_time < t <= test_time, test = t > test_time;
* evaluation negatives `<name>_{val,test}_ns.pkl`: a pickled dict (src, dst, t) -> negative
  destinations.  Pickles execute code when loaded, so they are read only with an explicit
  `allow_pickle=True` (the user vouching for their own download) and converted once into the
  `.npz` cache; the cache holds plain arrays only.

`load_tgb(name, root)` returns the arrays the rest of tgnx.data consumes, caching the parsed stream as
`<dir>/tgnx_<name>.npz` (src, dst, t, msg, train_end, val_end[, val_neg, test_neg]).
"""
from __future__ import annotations

import csv
import os

import numpy as np

TGB_NAMES = ("tgbl-wiki", "tgbl-review", "tgbl-coin", "tgbl-comment", "tgbl-flight")
VAL_RATIO, TEST_RATIO = 0.15, 0.15


def dataset_dir(name: str, root: str = "datasets") -> str:
    return os.path.join(root, name.replace("-", "_"))


def split_bounds(t: np.ndarray, val_ratio: float = VAL_RATIO, test_ratio: float = TEST_RATIO):
    """py-tgb generate_splits on time-sorted events: (train_end, val_end) event indices such that
    [0, train_end) = t <= val_time, [train_end, val_end) = val_time < t <= test_time, the rest test."""
    t = np.asarray(t)
    if t.size and np.any(np.diff(t) < 0):
        raise ValueError("TGB streams are time-sorted; got decreasing timestamps")
    val_time, test_time = np.quantile(t, [1.0 - val_ratio - test_ratio, 1.0 - test_ratio])
    return int(np.searchsorted(t, val_time, side="right")), int(np.searchsorted(t, test_time, side="right"))


def _raw_csv(d: str, name: str) -> str | None:
    for f in (f"{name}_edgelist_v2.csv", f"{name}_edgelist.csv", "ml_" + name + ".csv"):
        p = os.path.join(d, f)
        if os.path.exists(p):
            return p
    return None


def read_jodie_csv(path: str):
    """tgbl-wiki raw layout: user, item, timestamp, state_label, features..."""
    raw = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.float64, ndmin=2)
    u = raw[:, 0].astype(np.int64)
    i = raw[:, 1].astype(np.int64)
    t = raw[:, 2]
    msg = raw[:, 4:].astype(np.float32)
    if msg.shape[1] == 0:
        msg = np.ones((raw.shape[0], 1), dtype=np.float32)
    dst = i + int(u.max()) + 1
    return u, dst, t, msg


def read_edgelist_csv(path: str):
    """timestamp, source, destination[, weights...] with arbitrary node keys, relabelled to 0.. in order
    of first appearance (source before destination within an event)."""
    ids: dict = {}
    src, dst, ts, feats = [], [], [], []
    with open(path, newline="") as fh:
        rd = csv.reader(fh)
        next(rd)  # header
        for row in rd:
            if not row:
                continue
            ts.append(float(row[0]))
            s = ids.setdefault(row[1].strip(), len(ids))
            d = ids.setdefault(row[2].strip(), len(ids))
            src.append(s)
            dst.append(d)
            feats.append([float(x) for x in row[3:]])
    nf = len(feats[0]) if feats else 0
    msg = np.asarray(feats, dtype=np.float32).reshape(len(ts), nf) if nf else np.ones((len(ts), 1), np.float32)
    return np.asarray(src, np.int64), np.asarray(dst, np.int64), np.asarray(ts, np.float64), msg


def _negatives_from_pickle(path: str, src, dst, t, lo: int, hi: int) -> np.ndarray:
    import pickle  # only behind allow_pickle=True (see module docstring)
    with open(path, "rb") as fh:
        table = pickle.load(fh)
    rows = []
    for e in range(lo, hi):
        key = (int(src[e]), int(dst[e]), int(t[e]) if float(t[e]).is_integer() else float(t[e]))
        rows.append(np.asarray(table[key], dtype=np.int64))
    k = min(len(r) for r in rows) if rows else 0   # epoch_utils.py:45-49 truncates to the batch minimum
    return np.stack([r[:k] for r in rows]) if rows else np.zeros((0, 0), np.int64)


def uniform_negatives(dst: np.ndarray, lo: int, hi: int, k: int, seed: int = 0) -> np.ndarray:
    """Stand-in evaluation negatives when the TGB *_ns.pkl files are absent: k destinations per event of
    [lo, hi), uniform over the stream's destination set, redrawn where equal to the positive (TGB's own
    lists mix historical and random destinations; they cannot be regenerated here)."""
    rng = np.random.default_rng(seed)
    pool = np.unique(dst)
    out = pool[rng.integers(0, pool.size, size=(hi - lo, k))]
    pos = dst[lo:hi, None]
    for _ in range(8):
        bad = out == pos
        if not bad.any() or pool.size < 2:
            break
        out[bad] = pool[rng.integers(0, pool.size, size=int(bad.sum()))]
    return out.astype(np.int64)


def load_tgb(name: str, root: str = "datasets", allow_pickle: bool = False):
    """(src, dst, t, msg, train_end, val_end, negatives {val_neg, test_neg}) of a TGB dataset on disk, or
    None when `<root>/<name>/` holds neither the tgnx cache nor a raw edge list."""
    d = dataset_dir(name, root)
    cache = os.path.join(d, f"tgnx_{name}.npz")
    if os.path.exists(cache):
        z = np.load(cache, allow_pickle=False)
        negs = {k: z[k] for k in ("val_neg", "test_neg") if k in z.files}
        return z["src"], z["dst"], z["t"], z["msg"], int(z["train_end"]), int(z["val_end"]), negs
    raw = _raw_csv(d, name)
    if raw is None:
        return None
    src, dst, t, msg = read_jodie_csv(raw) if name == "tgbl-wiki" else read_edgelist_csv(raw)
    order = np.argsort(t, kind="stable")          # TGB streams are chronological
    src, dst, t, msg = src[order], dst[order], t[order], msg[order]
    tr, va = split_bounds(t)
    negs = {}
    for split, lo, hi in (("val", tr, va), ("test", va, len(t))):
        p = os.path.join(d, f"{name}_{split}_ns.pkl")
        if os.path.exists(p):
            if not allow_pickle:
                raise RuntimeError(f"{p} is a pickle (TGB negatives); pass allow_pickle=True to convert it once "
                                   f"into {cache}, or remove it to use generated negatives")
            negs[f"{split}_neg"] = _negatives_from_pickle(p, src, dst, t, lo, hi)
    np.savez(cache, src=src, dst=dst, t=t, msg=msg, train_end=tr, val_end=va, **negs)
    return src, dst, t, msg, tr, va, negs
