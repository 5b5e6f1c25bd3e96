"""ORACLE (test infrastructure only) — numpy restatement of `LastNeighborLoader`.

Follows /root/reference/neighbor_loader.py:
  __init__/reset_state  :16-24, :106-109   e_id = t = -1, cur_e_id = 0
  __call__              :26-50             gather [Q,K], mask e_id>=0 (row-major), unique, relabel
  insert                :52-104            both directions, dense [U,K] scatter, concat old+new,
                                            e_id top-K (neighbours follow e_id), t top-K separately

Canonical rule where the reference is undefined: when a node receives more than K
entries in one insert, the reference's survivors depend on an unstable sort
(:68) and a scatter with duplicate indices (:79); here the K largest e_id
survive.  Everywhere else this restatement is exact, which
tests/golden/sampler_*.npz checks.
"""
from __future__ import annotations

import numpy as np


class RefLastNeighborLoader:
    def __init__(self, num_nodes: int, size: int):
        self.size = int(size)
        self.num_nodes = int(num_nodes)
        self.neighbors = np.full((num_nodes, size), -1, dtype=np.int64)
        self.e_id = np.full((num_nodes, size), -1, dtype=np.int64)
        self.t = np.full((num_nodes, size), -1, dtype=np.float32)
        self._assoc = np.zeros(num_nodes, dtype=np.int64)
        self.reset_state()

    def reset_state(self):
        self.cur_e_id = 0
        self.e_id.fill(-1)
        self.t.fill(-1)

    def __call__(self, n_id: np.ndarray):
        n_id = np.asarray(n_id, dtype=np.int64)
        K = self.size
        nbr = self.neighbors[n_id]
        eid = self.e_id[n_id]
        tt = self.t[n_id]
        nodes = np.repeat(n_id, K).reshape(-1, K)
        mask = eid >= 0
        nbr, nodes, eid, tt = nbr[mask], nodes[mask], eid[mask], tt[mask]
        out_nid = np.unique(np.concatenate([n_id, nbr]))
        self._assoc[out_nid] = np.arange(out_nid.shape[0], dtype=np.int64)
        ei = np.stack([self._assoc[nbr], self._assoc[nodes]])
        return out_nid, ei, eid, tt

    def insert(self, src: np.ndarray, dst: np.ndarray, t: np.ndarray):
        src = np.asarray(src, dtype=np.int64)
        dst = np.asarray(dst, dtype=np.int64)
        t = np.asarray(t, dtype=np.float32)
        K = self.size
        B = src.shape[0]
        neighbors = np.concatenate([src, dst])
        nodes = np.concatenate([dst, src])
        e_id = np.tile(np.arange(self.cur_e_id, self.cur_e_id + B, dtype=np.int64), 2)
        tt = np.tile(t, 2)
        self.cur_e_id += B
        # group by node, newest (largest e_id) first
        order = np.lexsort((-e_id, nodes))
        nodes, neighbors, e_id, tt = nodes[order], neighbors[order], e_id[order], tt[order]
        uniq, start, inv = np.unique(nodes, return_index=True, return_inverse=True)
        U = uniq.shape[0]
        self._assoc[uniq] = np.arange(U, dtype=np.int64)
        rank = np.arange(nodes.shape[0]) - start[inv]
        keep = rank < K
        d_eid = np.full((U, K), -1, dtype=np.int64)
        d_t = np.full((U, K), -1, dtype=np.float32)
        d_nbr = np.full((U, K), -1, dtype=np.int64)
        d_eid[inv[keep], rank[keep]] = e_id[keep]
        d_t[inv[keep], rank[keep]] = tt[keep]
        d_nbr[inv[keep], rank[keep]] = neighbors[keep]
        c_eid = np.concatenate([self.e_id[uniq], d_eid], axis=1)
        c_t = np.concatenate([self.t[uniq], d_t], axis=1)
        c_nbr = np.concatenate([self.neighbors[uniq], d_nbr], axis=1)
        perm = np.argsort(-c_eid, axis=1, kind="stable")[:, :K]
        self.e_id[uniq] = np.take_along_axis(c_eid, perm, axis=1)
        self.neighbors[uniq] = np.take_along_axis(c_nbr, perm, axis=1)
        self.t[uniq] = -np.sort(-c_t, axis=1)[:, :K]
