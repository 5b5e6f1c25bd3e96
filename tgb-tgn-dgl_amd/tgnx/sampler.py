"""Drop-in `LastNeighborLoader` on the HIP ring kernels.

Same constructor, attributes (`neighbors`, `e_id`, `t`, `_assoc`, `size`,
`cur_e_id`) and methods (`__call__`, `insert`, `reset_state`) as
/root/reference/neighbor_loader.py:15-109; the work runs in libtgnx
(`tgnx_ring_sample` / `tgnx_ring_insert` / `tgnx_ring_reset`).
"""
from __future__ import annotations

import torch

from . import _lib


class LastNeighborLoader:
    def __init__(self, num_nodes: int, size: int, device=None):
        self.device = _lib.require_device(device)
        self.size = int(size)
        self.num_nodes = int(num_nodes)
        dev = self.device
        self.neighbors = torch.full((num_nodes, size), -1, dtype=torch.long, device=dev)
        self.e_id = torch.empty((num_nodes, size), dtype=torch.long, device=dev)
        self.t = torch.empty((num_nodes, size), dtype=torch.float, device=dev)
        self._assoc = torch.zeros(num_nodes, dtype=torch.long, device=dev)
        self._ws = torch.empty(0, dtype=torch.uint8, device=dev)
        self._ws_q = -1
        self._counts = torch.zeros(2, dtype=torch.long, device=dev)
        # bumped by every host-side change of the ring (reset_state / insert): an engine that prepared the
        # next batch from the ring (pipelined TGN step) re-prepares it when the version moved
        self.version = 0
        self.reset_state()

    # neighbor_loader.py:106-109
    def reset_state(self):
        self.cur_e_id = 0
        self.version += 1
        _lib.call("tgnx_ring_reset", _lib.ptr(self.e_id), _lib.ptr(self.t), self.num_nodes, self.size,
                  _lib.stream(self.device))

    def _workspace(self, q: int) -> torch.Tensor:
        if q > self._ws_q:
            q2 = max(q, 2 * max(self._ws_q, 0), 1024)
            nb = _lib.lib().tgnx_ring_sample_ws_bytes(self.num_nodes, q2)
            self._ws = torch.zeros(nb, dtype=torch.uint8, device=self.device)   # bitmap must start zeroed
            self._ws_q = q2
        return self._ws

    # neighbor_loader.py:26-50
    def __call__(self, n_id: torch.Tensor):
        n_id = torch.as_tensor(n_id).to(self.device, torch.long).contiguous()
        q = int(n_id.numel())
        K = self.size
        cap_n, cap_e = q * (1 + K), max(q * K, 1)
        out_nid = torch.empty(max(cap_n, 1), dtype=torch.long, device=self.device)
        out_ei = torch.empty(2 * cap_e, dtype=torch.long, device=self.device)
        out_eid = torch.empty(cap_e, dtype=torch.long, device=self.device)
        out_t = torch.empty(cap_e, dtype=torch.float, device=self.device)
        ws = self._workspace(q)
        _lib.call("tgnx_ring_sample", _lib.ptr(self.neighbors), _lib.ptr(self.e_id), _lib.ptr(self.t),
                  self.num_nodes, K, _lib.ptr(n_id), q, _lib.ptr(self._assoc), _lib.ptr(out_nid), _lib.ptr(out_ei),
                  _lib.ptr(out_eid), _lib.ptr(out_t), cap_n, cap_e, _lib.ptr(self._counts), _lib.ptr(ws),
                  ws.numel(), _lib.stream(self.device))
        M, E = self._counts.tolist()    # one D2H sync, like the reference's .unique()
        ei = out_ei.view(2, cap_e)[:, :E]
        return out_nid[:M], ei, out_eid[:E], out_t[:E]

    # neighbor_loader.py:52-104
    def insert(self, src: torch.Tensor, dst: torch.Tensor, t: torch.Tensor = None):
        src = torch.as_tensor(src).to(self.device, torch.long).contiguous()
        dst = torch.as_tensor(dst).to(self.device, torch.long).contiguous()
        t = torch.as_tensor(t).to(self.device, torch.float).contiguous()
        B = int(src.numel())
        cap = _lib.lib().tgnx_ring_insert_max_batch()
        if B > cap:
            raise RuntimeError(f"LastNeighborLoader.insert: batch {B} > {cap} supported by tgnx_ring_insert")
        _lib.call("tgnx_ring_insert", _lib.ptr(self.neighbors), _lib.ptr(self.e_id), _lib.ptr(self.t),
                  self.num_nodes, self.size, _lib.ptr(src), _lib.ptr(dst), _lib.ptr(t), B, self.cur_e_id,
                  _lib.ptr(self._assoc), _lib.stream(self.device))
        self.cur_e_id += B
        self.version += 1
