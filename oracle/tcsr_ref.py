"""ORACLE (test infrastructure only) — TGL's t-CSR graph and "recent" sampler, restated in numpy.

The reference loads DATA/<name>/ext_full.npz (utils.py:73) produced by tgb_gen_graph.py (README.md:5)
and builds TGL's C++ sampler with `setup.py build_ext` (README.md:2); neither the generator nor the
sampler sources are in /root/reference ([ext] TGL, unpinned).  Restated from TGL's published
gen_graph.py / sampler_core.cpp:
  gen_graph: per event row (src, dst, t, idx) append (dst, t, idx) to src's list and, with
             --add_reverse, (src, t, idx) to dst's list; indptr = cumulative lengths; each row sorted
             by time (np.argsort — here stable, ties kept in event order: the canonical choice).
  recent sampler: for a root (node, ts) the row position of the first entry with time >= ts is found
             by binary search and the num_neighbors entries before it are taken, newest first.
The event-id cutoff (entries with eid < cut) is the build's addition; at cut = a batch's first event
it equals LastNeighborLoader's ring row at that batch (neighbor_loader.py:52-104), which pins it to
the reference's own golden ring states (tests/test_tcsr_cpu.py).
"""
from __future__ import annotations

import numpy as np


def gen_graph(src, dst, t, num_nodes, add_reverse=True):
    src, dst = np.asarray(src, np.int64), np.asarray(dst, np.int64)
    t = np.asarray(t, np.float32)
    rows_i = [[] for _ in range(num_nodes)]
    rows_t = [[] for _ in range(num_nodes)]
    rows_e = [[] for _ in range(num_nodes)]
    for idx in range(src.shape[0]):
        s, d = int(src[idx]), int(dst[idx])
        rows_i[s].append(d); rows_t[s].append(t[idx]); rows_e[s].append(idx)
        if add_reverse:
            rows_i[d].append(s); rows_t[d].append(t[idx]); rows_e[d].append(idx)
    indptr = np.zeros(num_nodes + 1, np.int64)
    for i in range(num_nodes):
        indptr[i + 1] = indptr[i] + len(rows_i[i])
    indices = np.array([x for r in rows_i for x in r], np.int64)
    ts = np.array([x for r in rows_t for x in r], np.float32)
    eid = np.array([x for r in rows_e for x in r], np.int64)
    for i in range(num_nodes):
        a, b = indptr[i], indptr[i + 1]
        o = np.argsort(ts[a:b], kind="stable")
        indices[a:b], ts[a:b], eid[a:b] = indices[a:b][o], ts[a:b][o], eid[a:b][o]
    return indptr, indices, eid, ts


def sample_recent(indptr, indices, eid, ts, roots, K, cut_eid=None, cut_t=None):
    """(nbr, eid, ts, cnt) per root, newest first, -1 padded.  cut_eid: scalar or per-root array
    (eid < cut); cut_t: per-root array (ts < cut, TGL)."""
    roots = np.asarray(roots, np.int64)
    Q = roots.shape[0]
    on = np.full((Q, K), -1, np.int64)
    oe = np.full((Q, K), -1, np.int64)
    ot = np.full((Q, K), -1, np.float32)
    cnt = np.zeros(Q, np.int32)
    for q in range(Q):
        v = roots[q]
        a, b = indptr[v], indptr[v + 1]
        if cut_t is not None:
            p = a + np.searchsorted(ts[a:b], np.float32(cut_t[q]), side="left")
        else:
            c = cut_eid[q] if np.ndim(cut_eid) else cut_eid
            p = a + np.searchsorted(eid[a:b], c, side="left")
        w0 = max(a, p - K)
        n = p - w0
        cnt[q] = n
        on[q, :n] = indices[w0:p][::-1]
        oe[q, :n] = eid[w0:p][::-1]
        ot[q, :n] = ts[w0:p][::-1]
    return on, oe, ot, cnt
