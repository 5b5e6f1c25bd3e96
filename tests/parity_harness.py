"""Side-by-side runner: the HIP TGNN step vs the oracle's faithful per-block restatement.

Both start from the same parameters, the same synthetic stream, the same
dependency blocks and the same injected negatives; dropout is off (the two
RNG streams cannot be shared).  Used by tests/test_gpu_tgnn.py and by
__graft_entry__.smoke().
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import blocks_ref
from oracle.epoch_ref import eval_batch as ref_eval_batch
from oracle.epoch_ref import train_batch as ref_train_batch
from oracle.sampler_ref import RefLastNeighborLoader
from oracle.tgnn_ref import RefTGNN


class Pair:
    def __init__(self, N=400, E=1400, d=172, D=100, K=10, B=200, Kn_eval=20, seed=0, t_max=None, shape=None):
        from tgnx.engine import TgnnEngine
        from tgnx.model import TGNN, getOptimizer
        from tgnx.sampler import LastNeighborLoader
        from tgnx.synth import SHAPES, StreamShape, make_stream

        if shape is None:
            base = SHAPES["tgbl-wiki"]
            shape = StreamShape("parity", N, E, d, True, num_src=int(N * 0.85),
                                t_max=base.t_max if t_max is None else t_max)
            self.s = make_stream(shape, seed=seed)
        else:       # a named TGB shape (full node count), first E events of its stream
            self.s = make_stream(shape, seed=seed, num_events=E)
            N, d = self.s.num_nodes, self.s.shape.msg_dim
        self.B, self.K, self.D, self.d, self.N, self.Kn_eval = B, K, D, d, N, Kn_eval
        self.blk = blocks_ref.block_ids(self.s.src, self.s.dst, B)
        self.feats = torch.from_numpy(self.s.msg)
        torch.manual_seed(seed)
        self.ref = RefTGNN(d, D, N, feat_drop=0.0, attn_drop=0.0)
        self.ref_opt = torch.optim.Adam(self.ref.parameters(), lr=1e-4)
        self.ref_loader = RefLastNeighborLoader(N, K)
        sd = {k: v.detach().clone() for k, v in self.ref.named_parameters()}
        self.model = TGNN(d, D, N, "cuda", ring=K, max_batch=B, max_neg=Kn_eval, feat_drop=0.0, attn_drop=0.0)
        self.model.load_reference_state(sd)
        self.opt = getOptimizer({"gnn": self.model}, 1e-4)
        self.loader = LastNeighborLoader(N, K, device="cuda")
        self.eng = TgnnEngine(self.model, self.loader, self.feats, self.opt, max_neg=Kn_eval, seed=seed)
        self.rng = np.random.default_rng(seed + 99)
        self.pos = 0

    def _batch(self, B):
        sl = slice(self.pos, self.pos + B)
        self.pos += B
        s = self.s
        t32 = s.t[sl].astype(np.float32)
        return (torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl]), torch.from_numpy(t32),
                torch.from_numpy(s.msg[sl]), torch.from_numpy(self.blk[sl]))

    def prefill(self, n_events, chunk=None):
        """Advance both rings (and the e_id counter) over the next `n_events` events, batch by batch,
        without training: a later step then samples full rings, as mid-epoch (`neighbor_loader.insert`,
        epoch_utils.py:300)."""
        chunk = chunk or self.B
        end = self.pos + n_events
        while self.pos < end:
            n = min(chunk, end - self.pos)
            sl = slice(self.pos, self.pos + n)
            self.pos += n
            t32 = self.s.t[sl].astype(np.float32)
            self.ref_loader.insert(self.s.src[sl], self.s.dst[sl], t32)
            self.loader.insert(torch.from_numpy(self.s.src[sl]), torch.from_numpy(self.s.dst[sl]),
                               torch.from_numpy(t32))

    def train_step(self):
        src, dst, t, msg, blk = self._batch(self.B)
        neg = torch.from_numpy(self.rng.choice(self.s.dst_nodes, size=src.shape[0]))
        ref_loss, ref_pos, ref_neg = ref_train_batch(self.ref, self.ref_opt, self.ref_loader, self.feats, src, dst,
                                                     neg, t, msg, blk)
        pos, negl, _ = self.eng.train_batch(src, dst, t, msg, blk, neg=neg, dropout=False)
        torch.cuda.synchronize()
        self.eng.check()
        order = np.argsort(blk.numpy(), kind="stable")      # reference rows are in block order
        return dict(ref_loss=float(ref_loss), loss=float(self.model.grad_flat[-1]),
                    ref_pos=ref_pos.view(-1).numpy(), pos=pos.cpu().numpy()[order],
                    ref_neg=ref_neg.view(-1).numpy(), neg=negl.cpu().numpy()[order])

    def eval_step(self, quirk=True):
        src, dst, t, msg, blk = self._batch(self.B)
        neg2d = np.stack([self.rng.choice(self.s.dst_nodes, size=self.Kn_eval, replace=False)
                          for _ in range(src.shape[0])])
        neg2d = torch.from_numpy(neg2d.astype(np.int64))
        self.ref.eval()
        ref_mrr, ref_pos, ref_neg = ref_eval_batch(self.ref, self.ref_loader, self.feats, src, dst, neg2d, t, msg,
                                                   blk)
        pos, negl, mrr = self.eng.eval_batch(src, dst, t, msg, blk, neg2d, tile_quirk=quirk)
        torch.cuda.synchronize()
        self.eng.check()
        return dict(ref_mrr=ref_mrr, mrr=float(mrr), ref_pos=ref_pos.numpy(), pos=pos.cpu().numpy(),
                    ref_neg=ref_neg.numpy(), neg=negl.cpu().numpy())

    def sync_from_ref(self):
        """Copy the oracle's parameters and Adam moments into the HIP model, so the next step is
        compared from identical state.  Needed at wiki time scales: cos(w*dt + b) with dt ~ 1e6 makes
        the model chaotic in te_w (1 ulp of w = 1.0 turns the phase by ~0.16 rad), so any two fp32
        implementations drift apart over steps; each step's kernels are still checked exactly."""
        with torch.no_grad():
            for k, p in self.ref.named_parameters():
                if not p.requires_grad:
                    continue
                off, n, _ = self.model._views[k]
                self.model.flat[off:off + n].copy_(p.detach().reshape(-1))
                st = self.ref_opt.state.get(p, {})
                if "exp_avg" in st:
                    self.eng.adam_m[off:off + n].copy_(st["exp_avg"].reshape(-1))
                    self.eng.adam_v[off:off + n].copy_(st["exp_avg_sq"].reshape(-1))
        self._ill = {}

    def ref_grads(self):
        return {k: p.grad.detach().numpy() for k, p in self.ref.named_parameters() if p.grad is not None}

    def gpu_grads(self):
        return {k: v.detach().cpu().numpy() for k, v in self.model.grads_by_name().items()}

    def param_diff(self, rel_floor=1e-3):
        """Max |param_gpu - param_ref| after the optimizer step, split by gradient conditioning.

        Adam's first steps move a parameter by ~lr * g/|g|, so elements whose gradient is at the
        fp32 cancellation floor (|g| < rel_floor * max|g| of the tensor, e.g. attn_r: er shifts a
        whole softmax) may move by +-lr in either implementation; once ill, an element stays excluded
        (the momentum carries it).  Returns (well, all)."""
        well, allv = {}, {}
        if not hasattr(self, "_ill"):
            self._ill = {}
        for k, p in self.ref.named_parameters():
            if not p.requires_grad or p.grad is None:
                continue
            off, n, shape = self.model._views[k]
            g = self.model.flat[off:off + n].view(shape).cpu().numpy()
            d = np.abs(g - p.detach().numpy())
            gr = np.abs(p.grad.detach().numpy())
            ill = gr <= rel_floor * max(gr.max(), 1e-30)
            self._ill[k] = ill | self._ill.get(k, np.zeros_like(ill))   # Adam momentum carries history
            mask = ~self._ill[k]
            well[k] = float(d[mask].max()) if mask.any() else 0.0
            allv[k] = float(d.max())
        return well, allv

    def state_equal(self):
        eid = self.loader.e_id.cpu().numpy()
        ok = np.array_equal(eid, self.ref_loader.e_id)
        ok &= np.array_equal(self.loader.t.cpu().numpy(), self.ref_loader.t)
        nb = self.loader.neighbors.cpu().numpy()
        ok &= np.array_equal(nb[eid >= 0], self.ref_loader.neighbors[self.ref_loader.e_id >= 0])
        ta_ok = np.array_equal(self.model.time_assoc.cpu().numpy(), self.ref.time_assoc.numpy())
        return bool(ok), bool(ta_ok)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))
