"""t-CSR temporal graph and the "recent" neighbour sampler on the device (include/tgnx.h tgnx_tcsr_*).

TCSR holds TGL's ext_full.npz arrays (indptr, indices, eid, ts — the file utils.py:73 loads; the
generator tgb_gen_graph.py and TGL's C++ sampler are absent from the reference) as device tensors:

    g = TCSR.build(src, dst, t, num_nodes)              # on the device (stable radix sort)
    g.save_npz("DATA/tgbl-wiki/ext_full.npz"); g = TCSR.load_npz(path, device)
    nbr, eid, ts, cnt = g.sample_recent(roots, K, cut_eid=batch_start)   # == LastNeighborLoader ring rows
    nbr, eid, ts, cnt = g.sample_recent(roots, K, cut_t=root_times)      # TGL: strictly before each root's t
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _p(t):
    return 0 if t is None else t.data_ptr()


class TCSR:
    def __init__(self, indptr, indices, eid, ts, chronological: bool = True):
        self.indptr, self.indices, self.eid, self.ts = indptr, indices, eid, ts
        self.num_nodes = int(indptr.numel()) - 1
        self.chronological = bool(chronological)

    @property
    def device(self):
        return self.indptr.device

    @classmethod
    def build(cls, src, dst, t, num_nodes: int, add_reverse: bool = True, device=None) -> "TCSR":
        dev = _lib.require_device(device if device is not None else (src.device if torch.is_tensor(src) else None))
        src = torch.as_tensor(src).to(dev, torch.long).contiguous()
        dst = torch.as_tensor(dst).to(dev, torch.long).contiguous()
        t = torch.as_tensor(t).to(dev, torch.float32).contiguous()
        E = int(src.numel())
        nnz = 2 * E if add_reverse else E
        indptr = torch.empty(num_nodes + 1, dtype=torch.long, device=dev)
        indices = torch.empty(max(nnz, 1), dtype=torch.long, device=dev)
        eid = torch.empty(max(nnz, 1), dtype=torch.long, device=dev)
        ts = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        nb = _lib.lib().tgnx_tcsr_build_ws_bytes(E, int(add_reverse))
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        chrono = ctypes.c_int32(1)
        _lib.call("tgnx_tcsr_build", _p(src), _p(dst), _p(t), E, num_nodes, int(add_reverse), _p(indptr), _p(indices),
                  _p(eid), _p(ts), ctypes.byref(chrono), _p(ws), ctypes.c_size_t(nb), _lib.stream(dev))
        return cls(indptr, indices[:nnz], eid[:nnz], ts[:nnz], bool(chrono.value))

    def save_npz(self, path: str) -> None:
        np.savez(path, indptr=self.indptr.cpu().numpy(), indices=self.indices.cpu().numpy(),
                 eid=self.eid.cpu().numpy(), ts=self.ts.cpu().numpy())

    @classmethod
    def load_npz(cls, path: str, device=None) -> "TCSR":
        dev = _lib.require_device(device)
        z = np.load(path)                      # allow_pickle=False: plain arrays only
        f = lambda k, dt: torch.from_numpy(np.ascontiguousarray(z[k])).to(dev, dt)  # noqa: E731
        g = cls(f("indptr", torch.long), f("indices", torch.long), f("eid", torch.long), f("ts", torch.float32))
        ts = z["ts"]
        g.chronological = bool(np.all([np.all(np.diff(ts[a:b]) >= 0) for a, b in zip(z["indptr"][:-1], z["indptr"][1:])]))
        return g

    def sample_recent(self, roots, K: int, cut_eid=None, cut_t=None):
        """K most recent entries of each root's row before the cutoff, newest first.  cut_eid: int (all
        roots) or LongTensor[Q] — eid < cut; cut_t: FloatTensor[Q] — ts < cut_t (TGL).  Returns
        (nbr [Q,K], eid [Q,K], ts [Q,K], cnt [Q]); empty slots hold -1."""
        dev = self.device
        roots = torch.as_tensor(roots).to(dev, torch.long).contiguous()
        Q = int(roots.numel())
        nbr = torch.empty(Q, K, dtype=torch.long, device=dev)
        eid = torch.empty(Q, K, dtype=torch.long, device=dev)
        ts = torch.empty(Q, K, dtype=torch.float32, device=dev)
        cnt = torch.empty(Q, dtype=torch.int32, device=dev)
        if cut_t is not None:
            if not self.chronological:
                raise ValueError("time cutoff on a t-CSR whose rows are not time-sorted (non-chronological stream)")
            ct = torch.as_tensor(cut_t).to(dev, torch.float32).contiguous()
            mode, ce, ce_all = 1, None, 0
        else:
            ct = None
            mode = 0
            if torch.is_tensor(cut_eid) or isinstance(cut_eid, np.ndarray):
                ce, ce_all = torch.as_tensor(cut_eid).to(dev, torch.long).contiguous(), 0
            else:
                ce, ce_all = None, int(cut_eid if cut_eid is not None else np.iinfo(np.int64).max)
        _lib.call("tgnx_tcsr_sample", _p(self.indptr), _p(self.indices), _p(self.eid), _p(self.ts), self.num_nodes, K,
                  _p(roots), Q, mode, _p(ce), ce_all, _p(ct), _p(nbr), _p(eid), _p(ts), _p(cnt), _lib.stream(dev))
        return nbr, eid, ts, cnt
