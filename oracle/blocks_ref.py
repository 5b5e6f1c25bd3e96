"""ORACLE (test infrastructure only) — restatement of dependency-block assignment.

Follows /root/reference/dependencyGraph.py:8-28 (`get_block`) and :33-49
(`dependecyAwareBatch`, flat=True): per batch, a fresh map node -> last block;
each edge in batch order gets block = 1 + max(last[src], last[dst]) (missing = -1),
then last[src] = last[dst] = block.  Pure-Python loop: small cases only.
Pinned by tests/golden/blocks.npz.
"""
from __future__ import annotations

import numpy as np


def get_block(src, dst) -> list[int]:
    last: dict[int, int] = {}
    out = []
    for a, b in zip(np.asarray(src).tolist(), np.asarray(dst).tolist()):
        blk = max(last.get(a, -1), last.get(b, -1)) + 1
        last[a] = blk
        last[b] = blk
        out.append(blk)
    return out


def block_ids(src, dst, batch_size: int) -> np.ndarray:
    src = np.asarray(src)
    dst = np.asarray(dst)
    out = []
    for s in range(0, src.shape[0], batch_size):
        out.extend(get_block(src[s:s + batch_size], dst[s:s + batch_size]))
    return np.asarray(out, dtype=np.int64)
