"""Drop-in `NegLinkSamplerDest` (neg_sampler.py:3-23) on the HIP counter-based sampler.

Same draw distribution as the reference — uniform over the unique destinations,
redrawn where it hits the positive — but from a counter-based stream keyed by
(seed, call, position), so a step is replayable and graph-capturable.  The
reference's unseeded torch CPU draw cannot be reproduced on the device; parity
tests inject negatives instead (SURVEY.md §7 hard part 4).
"""
from __future__ import annotations

import torch

from . import _lib


class NegLinkSamplerDest:
    def __init__(self, dst_nodes: torch.Tensor, device=None, seed: int = 0):
        self.device = _lib.require_device(device)
        self.dst_nodes = torch.as_tensor(dst_nodes, dtype=torch.long).to(self.device).contiguous()
        self.seed = int(seed)
        self._offset = 0

    def sample(self, pos_dst: torch.Tensor) -> torch.Tensor:
        pos = pos_dst.to(self.device, torch.long).contiguous()
        out = torch.empty_like(pos)
        self.sample_into(pos, out)
        return out

    def sample_into(self, pos: torch.Tensor, out: torch.Tensor, offset: int | None = None) -> None:
        B = int(pos.numel())
        off = self._offset if offset is None else int(offset)
        _lib.call("tgnx_neg_sample", _lib.ptr(self.dst_nodes), self.dst_nodes.numel(), _lib.ptr(pos), B,
                  self.seed, off, _lib.ptr(out), _lib.stream(self.device))
        if offset is None:
            self._offset += B
