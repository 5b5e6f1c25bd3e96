"""Synthetic TGB-shaped temporal event streams.

TGB datasets cannot be downloaded here (no network), so every benchmark and
parity test runs on a seeded synthetic stream with the published shape of the
dataset it stands in for: node count, event count, edge-feature width,
bipartite or not, timestamp scale, and a chronological 70/15/15 split
(the split `utils.py:30-40` takes from TGB's masks).

Events are sorted by time, so an event's row index is its global e_id: the
running counter `LastNeighborLoader.insert` assigns (`neighbor_loader.py:59-64`)
equals the row of `data.msg` that `epoch_utils.py:224` gathers, because val
continues the train split without a reset.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass(frozen=True)
class StreamShape:
    name: str
    num_nodes: int
    num_events: int
    msg_dim: int
    bipartite: bool
    num_src: int = 0            # bipartite: ids [0, num_src) are sources
    zipf_src: float = 1.6
    zipf_dst: float = 1.3
    t_max: int = 2_678_373      # wiki: integer seconds from 0
    t_base: float = 0.0         # unix-scale streams add ~9.3e8
    num_neg_eval: int = 999
    mail_combine: str = "last"


SHAPES = {
    "tgbl-wiki": StreamShape("tgbl-wiki", 9_227, 157_474, 172, True, num_src=8_227),
    "tgbl-review": StreamShape("tgbl-review", 352_637, 4_873_540, 1, True, num_src=352_637 - 1_000,
                               t_max=150_000_000, t_base=9.3e8, num_neg_eval=100, mail_combine="mean"),
    "tgbl-coin": StreamShape("tgbl-coin", 638_486, 22_809_486, 1, False, t_max=50_000_000,
                             t_base=1.5e9, num_neg_eval=100),
    "tgbl-comment": StreamShape("tgbl-comment", 994_790, 44_314_507, 2, False, t_max=100_000_000,
                                t_base=1.2e9, num_neg_eval=100),
}


def _zipf_ids(rng: np.random.Generator, n: int, a: float, size: int) -> np.ndarray:
    """Finite Zipf(a) over n ids (p_k ∝ k^-a, k=1..n) under a random id permutation."""
    p = np.arange(1, n + 1, dtype=np.float64) ** (-a)
    p /= p.sum()
    ranks = rng.choice(n, size=size, p=p)
    perm = rng.permutation(n)
    return perm[ranks]


@dataclass
class TemporalStream:
    """Host arrays of one synthetic stream (the PyG TemporalData fields)."""
    shape: StreamShape
    src: np.ndarray        # int64 [E]
    dst: np.ndarray        # int64 [E]
    t: np.ndarray          # float64 [E] (cast to fp32 at batching, temporal_dataset.py:42,53)
    msg: np.ndarray        # float32 [E, d]
    train_end: int
    val_end: int
    dst_nodes: np.ndarray = field(default=None)   # sorted unique destinations

    @property
    def num_nodes(self) -> int:
        return self.shape.num_nodes

    @property
    def num_events(self) -> int:
        return int(self.src.shape[0])

    def split(self, which: str) -> slice:
        if which == "train":
            return slice(0, self.train_end)
        if which == "val":
            return slice(self.train_end, self.val_end)
        if which == "test":
            return slice(self.val_end, self.num_events)
        raise ValueError(which)


def make_stream(shape: StreamShape | str, seed: int = 0, num_events: int | None = None,
                num_nodes: int | None = None, msg_dim: int | None = None) -> TemporalStream:
    """Generate a chronological stream with `shape`'s statistics (optionally scaled down)."""
    if isinstance(shape, str):
        shape = SHAPES[shape]
    if num_events is not None or num_nodes is not None or msg_dim is not None:
        n = num_nodes or shape.num_nodes
        ns = shape.num_src
        if shape.bipartite:
            ns = max(1, int(round(n * shape.num_src / shape.num_nodes)))
            ns = min(ns, n - 1)
        shape = StreamShape(shape.name, n, num_events or shape.num_events,
                            shape.msg_dim if msg_dim is None else msg_dim, shape.bipartite, ns,
                            shape.zipf_src, shape.zipf_dst, shape.t_max, shape.t_base,
                            shape.num_neg_eval, shape.mail_combine)
    rng = np.random.default_rng(seed)
    E = shape.num_events
    if shape.bipartite:
        src = _zipf_ids(rng, shape.num_src, shape.zipf_src, E)
        dst = shape.num_src + _zipf_ids(rng, shape.num_nodes - shape.num_src, shape.zipf_dst, E)
    else:
        src = _zipf_ids(rng, shape.num_nodes, shape.zipf_src, E)
        dst = _zipf_ids(rng, shape.num_nodes, shape.zipf_dst, E)
    t = np.sort(rng.integers(0, shape.t_max + 1, size=E)).astype(np.float64) + shape.t_base
    msg = rng.random((E, shape.msg_dim), dtype=np.float32)
    train_end = int(round(0.70 * E))
    val_end = int(round(0.85 * E))
    s = TemporalStream(shape, src.astype(np.int64), dst.astype(np.int64), t, msg, train_end, val_end)
    s.dst_nodes = np.unique(s.dst)
    return s


def eval_negatives(stream: TemporalStream, split: str, num_neg: int | None = None,
                   seed: int = 1, limit: int | None = None) -> np.ndarray:
    """Per-positive eval negatives drawn from the destination set, excluding the positive.

    Stands in for TGB's precomputed `*_ns.pkl` (`epoch_utils.py:43`): Long[E_split, num_neg]
    (the split's first `limit` events only, if given).
    """
    sl = stream.split(split)
    pos = stream.dst[sl]
    if limit is not None:
        pos = pos[:limit]
    k = stream.shape.num_neg_eval if num_neg is None else num_neg
    rng = np.random.default_rng(seed + (0 if split == "val" else 7919))
    cand = stream.dst_nodes
    idx = rng.integers(0, cand.shape[0] - 1, size=(pos.shape[0], k))
    # skip the positive's own slot so every draw is a true negative
    pos_rank = np.searchsorted(cand, pos)
    idx = idx + (idx >= pos_rank[:, None])
    return cand[np.minimum(idx, cand.shape[0] - 1)].astype(np.int64)
