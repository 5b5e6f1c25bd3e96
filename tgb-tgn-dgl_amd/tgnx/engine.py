"""Host orchestration of the fused TGNN step (one process per GPU).

A train step (epoch_utils.py:186-315) is two C-ABI calls on the current HIP stream:
  tgnx_tgnn_train_fwd_bwd  negatives, assembly, forward, predictor + BCE, backward -> flat grads
  [torch.distributed.all_reduce(grads) when world_size > 1 — RCCL over xGMI]
  tgnx_tgnn_train_update   Adam, ring insert of the whole (global) batch, time_assoc
An eval step (epoch_utils.py:28-157) is one call (tgnx_tgnn_eval_step).  Batch
geometry lives in a device control block, so steps never synchronise the host
and a sequence of them can be captured in a HIP graph (tgnx.graph).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .model import TGNN, FusedAdam, TgnnConfig

CTL = dict(BATCH_START=0, CUR_EID=1, B=2, GEN=3, ADAM_T=4, S=5, E=6, LO=7, HI=8, SEED=9, NB=10, ERR=11, LOSS=12)

P = ctypes.c_void_p


class TgnnBuffers(ctypes.Structure):
    _fields_ = [("ev_src", P), ("ev_dst", P), ("ev_t", P), ("ev_blk", P), ("ev_msg", P), ("neg", P),
                ("dst_nodes", P), ("n_dst", ctypes.c_int64), ("feat", P), ("nbr", P), ("eid", P), ("rt", P),
                ("assoc", P), ("time_assoc", P), ("memory", P), ("params", P), ("grads", P), ("adam_m", P),
                ("adam_v", P), ("ctl", P), ("out_pos", P), ("out_neg", P), ("mrr", P), ("ws", P), ("node_map", P),
                ("out_ev", P)]




def _p(t):
    return 0 if t is None else t.data_ptr()


class TgnnEngine:
    """Owns the device workspace of one model + one neighbour ring."""

    def __init__(self, model: TGNN, loader, feat: torch.Tensor, optimizer: FusedAdam | None,
                 dst_nodes: torch.Tensor | None = None, max_neg: int | None = None, seed: int = 0,
                 rank: int = 0, world: int = 1):
        self.model, self.loader, self.opt = model, loader, optimizer
        self.dev = model.device
        cfg = model.cfg
        if max_neg is not None and max_neg > cfg.max_neg:
            cfg.max_neg = int(max_neg)
        if cfg.ring != loader.size:
            cfg.ring = loader.size
        self.cfg = cfg
        self.feat = feat.to(self.dev, torch.float32).contiguous()
        nb = _lib.lib().tgnx_tgnn_ws_bytes(ctypes.byref(cfg))
        if nb == 0:
            raise RuntimeError(f"tgnx_tgnn_ws_bytes: invalid config: {_lib.lib().tgnx_last_error().decode()}")
        self.ws = torch.zeros(nb, dtype=torch.uint8, device=self.dev)
        self.node_map = torch.zeros(4 * cfg.num_nodes, dtype=torch.int32, device=self.dev)
        self.ctl = torch.zeros(24, dtype=torch.int64, device=self.dev)   # TGNX_CTL_WORDS
        cap = cfg.max_batch * max(cfg.max_neg, 1)
        self.out_pos = torch.zeros(cfg.max_batch, dtype=torch.float32, device=self.dev)
        self.out_neg = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.mrr = torch.zeros(1 << 16, dtype=torch.float64, device=self.dev)
        self.dst_nodes = None if dst_nodes is None else dst_nodes.to(self.dev, torch.long).contiguous()
        self.seed, self.rank, self.world = int(seed), int(rank), int(world)
        if optimizer is None:
            self.adam_m = torch.zeros_like(model.flat)
            self.adam_v = torch.zeros_like(model.flat)
        else:
            self.adam_m, self.adam_v = optimizer.exp_avg, optimizer.exp_avg_sq
        self._neg_scratch = None
        self.out_ev = None    # optional per-event train-logit log (tgnx_tgnn_buffers.out_ev)
        self.fold_cursor = True
        self.fuse_adam = True

    # ------------------------------------------------------------------ plumbing
    def _buffers(self, src, dst, t, blk, msg, neg) -> TgnnBuffers:
        m, ld = self.model, self.loader
        b = TgnnBuffers()
        b.ev_src, b.ev_dst, b.ev_t, b.ev_blk, b.ev_msg = _p(src), _p(dst), _p(t), _p(blk), _p(msg)
        b.neg = neg if isinstance(neg, int) else _p(neg)
        b.dst_nodes = _p(self.dst_nodes)
        b.n_dst = 0 if self.dst_nodes is None else self.dst_nodes.numel()
        b.feat = _p(self.feat)
        b.nbr, b.eid, b.rt, b.assoc = _p(ld.neighbors), _p(ld.e_id), _p(ld.t), _p(ld._assoc)
        b.time_assoc, b.memory = _p(m.time_assoc), _p(m.memory.memory)
        b.params, b.grads, b.adam_m, b.adam_v = _p(m.flat), _p(m.grad_flat), _p(self.adam_m), _p(self.adam_v)
        b.ctl, b.out_pos, b.out_neg, b.mrr = _p(self.ctl), _p(self.out_pos), _p(self.out_neg), _p(self.mrr)
        b.ws, b.node_map = _p(self.ws), _p(self.node_map)
        b.out_ev = _p(self.out_ev)
        return b

    def _stream(self):
        return _lib.stream(self.dev)

    def advance(self, mode, batch_start=0, B=0, cur_e_id=0, split_lo=0, split_hi=0, batch=1, train=True):
        _lib.call("tgnx_tgnn_advance", _p(self.ctl), mode, batch_start, B, cur_e_id, split_lo, split_hi, batch,
                  self.rank, self.world, self.seed, 1 if train else 0, self._stream())

    def _allreduce_grads(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(self.model.grad_flat)

    # ------------------------------------------------------------------ explicit (per-batch tensors)
    @staticmethod
    def _dev_batch(dev, src, dst, t, msg, blk):
        f = lambda x, dt: torch.as_tensor(x).to(dev, dt, non_blocking=True).contiguous()  # noqa: E731
        return f(src, torch.long), f(dst, torch.long), f(t, torch.float32), f(msg, torch.float32), f(blk, torch.long)

    def train_batch(self, src, dst, t, msg, blk, neg=None, dropout=True, update=True):
        """One train iteration on an explicit batch (epoch_utils.py:194-304).  update=False stops
        after the gradients (no all-reduce, no Adam; the ring insert / time_assoc update of the batch
        already happened once the forward had read them): see apply_update()."""
        self.finish()   # (a resident step's deferred update first: this step overwrites the reduced gradients)
        dev = self.dev
        src, dst, t, msg, blk = self._dev_batch(dev, src, dst, t, msg, blk)
        B = int(src.numel())
        gen_neg = neg is None
        if gen_neg:
            neg = torch.empty(B, dtype=torch.long, device=dev)
        else:
            neg = torch.as_tensor(neg).to(dev, torch.long).reshape(-1).contiguous()
        self.advance(0, 0, B, self.loader.cur_e_id, train=True)
        buf = self._buffers(src, dst, t, blk, msg, neg)
        _lib.call("tgnx_tgnn_train_fwd_bwd", ctypes.byref(self.cfg), ctypes.byref(buf), 1 if gen_neg else 0,
                  1 if (dropout and self.model.training) else 0, self._stream())
        self._keep = (src, dst, t, msg, blk, neg)   # keep alive until the stream consumes them
        self._pending = (buf, B)
        if update:
            self.apply_update()
        return self.out_pos[:B], self.out_neg[:B], neg

    def apply_update(self, allreduce=True):
        """All-reduce (world > 1) and Adam for the last train_batch."""
        buf, B = self._pending
        if allreduce:
            self._allreduce_grads()
        _lib.call("tgnx_tgnn_train_update", ctypes.byref(self.cfg), ctypes.byref(buf), self._stream())
        self.loader.cur_e_id += B

    def eval_batch(self, src, dst, t, msg, blk, neg2d, tile_quirk=True):
        """One eval iteration (epoch_utils.py:28-157); returns (pos[B], neg[B,K'], mrr) in block order."""
        dev = self.dev
        src, dst, t, msg, blk = self._dev_batch(dev, src, dst, t, msg, blk)
        neg2d = torch.as_tensor(neg2d).to(dev, torch.long).contiguous()
        B, Kn = neg2d.shape
        if Kn > self.cfg.max_neg:
            raise RuntimeError(f"eval_batch: {Kn} negatives per event > max_neg={self.cfg.max_neg}")
        self.advance(0, 0, B, self.loader.cur_e_id, train=False)
        buf = self._buffers(src, dst, t, blk, msg, neg2d)
        _lib.call("tgnx_tgnn_eval_step", ctypes.byref(self.cfg), ctypes.byref(buf), Kn, 1 if tile_quirk else 0,
                  self._stream())
        self.loader.cur_e_id += B
        self._keep = (src, dst, t, msg, blk, neg2d)
        nb = int(self.ctl[CTL["NB"]])
        return self.out_pos[:B], self.out_neg[:B * Kn].view(B, Kn), self.mrr[(nb - 1) & 0xFFFF]

    # ------------------------------------------------------------------ resident (events in HBM)
    def bind_resident(self, src, dst, t, blk, msg, neg_buf, split_lo, split_hi, batch, dropout=True):
        """Point the step at device-resident event arrays (global event index = row): the batch
        cursor lives in the control block, so a step is three launches of C calls and no host sync."""
        self.finish()        # (a pending update of the previous binding's last step)
        self._group = None   # (a step group captured for a previous binding)
        self._res_keep = (src, dst, t, blk, msg, neg_buf)
        self._res_buf = self._buffers(src, dst, t, blk, msg, neg_buf)
        self._res = (int(split_lo), int(split_hi), int(batch))
        self._res_drop = 1 if (dropout and self.model.training) else 0
        L = _lib.lib()
        self._f = (L.tgnx_tgnn_advance, L.tgnx_tgnn_train_fwd_bwd, L.tgnx_tgnn_train_update)
        # the batch cursor folded into the step's first launch (tgnx_tgnn_train_fwd_bwd_resident: one launch fewer);
        # fold_cursor = False keeps tgnx_tgnn_advance + tgnx_tgnn_train_fwd_bwd (same results)
        self._fold = self.fold_cursor and hasattr(L, "tgnx_tgnn_train_fwd_bwd_resident")
        # world 1: Adam and the loss sum folded into the step's gradient expansion (tgnx_tgnn_train_step_resident: no
        # tgnx_tgnn_train_update launch); fuse_adam = False keeps the separate update
        self._fused = self._fold and self.fuse_adam and self.world == 1 and hasattr(L, "tgnx_tgnn_train_step_resident")
        # ... and deferred: each step's update runs in the next step's first launch (finish() applies the last one)
        self._defer = self._fused and hasattr(L, "tgnx_tgnn_apply_pending")
        self._cfg_ref = ctypes.byref(self.cfg)
        self._buf_ref = ctypes.byref(self._res_buf)
        self._ctl_p = ctypes.c_void_p(self.ctl.data_ptr())

    def begin_epoch(self):
        """epoch_utils.py:175 — neighbor_loader.reset_state() at every train epoch; batch cursor to 0."""
        self.loader.reset_state()
        self.ctl[CTL["NB"]] = 0

    def _resident_fwd_bwd(self, st):
        adv, fb, _ = self._f
        lo, hi, batch = self._res
        if self._fused:
            return _lib.lib().tgnx_tgnn_train_step_resident(self._cfg_ref, self._buf_ref, lo, hi, batch, self.seed,
                                                           self._res_drop, st)
        if self._fold:
            return _lib.lib().tgnx_tgnn_train_fwd_bwd_resident(self._cfg_ref, self._buf_ref, lo, hi, batch, self.rank,
                                                              self.world, self.seed, self._res_drop, st)
        rc = adv(self._ctl_p, 1, 0, 0, 0, lo, hi, batch, self.rank, self.world, self.seed, 1, st)
        return rc | fb(self._cfg_ref, self._buf_ref, 1, self._res_drop, st)

    def resident_train_step(self):
        up = self._f[2]
        st = self._stream()
        rc = self._resident_fwd_bwd(st)
        if rc:
            raise RuntimeError(f"tgnx resident step failed: {_lib.lib().tgnx_last_error().decode()}")
        if self._fused:
            return
        self._allreduce_grads()
        if up(self._cfg_ref, self._buf_ref, st):
            raise RuntimeError(f"tgnx resident update failed: {_lib.lib().tgnx_last_error().decode()}")

    def finish(self):
        """Apply the update the last resident step left pending (world 1: tgnx_tgnn_train_step_resident defers each
        step's gradient expansion + Adam into the next step's first launch).  Call before reading the parameters
        or the Adam moments; the drop-in train() does, and an eval step applies a pending update itself."""
        if getattr(self, "_defer", False):
            if _lib.lib().tgnx_tgnn_apply_pending(self._cfg_ref, self._buf_ref, self._stream()):
                raise RuntimeError(f"tgnx apply_pending failed: {_lib.lib().tgnx_last_error().decode()}")

    def capture_resident(self, steps_per_graph: int = 1):
        """Capture `steps_per_graph` resident train steps into HIP graphs (torch.cuda.CUDAGraph).
        Every kernel reads its batch from the device control block, so replaying a graph advances
        through consecutive batches.  world > 1: the gradient all-reduce stays eager between a
        captured forward/backward graph and a captured update graph."""
        up = self._f[2]
        cfg, buf = self._cfg_ref, self._buf_ref

        def pre():
            rc = self._resident_fwd_bwd(self._stream())
            if rc:
                raise RuntimeError(_lib.lib().tgnx_last_error().decode())

        def post():
            if self._fused:
                return
            if up(cfg, buf, self._stream()):
                raise RuntimeError(_lib.lib().tgnx_last_error().decode())

        # capture runs the work once? no: capture only records; keep the cursor unchanged
        torch.cuda.synchronize(self.dev)
        saved = self.ctl.clone()
        sstream = torch.cuda.Stream(self.dev)
        sstream.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(sstream):   # warm the caching allocator on the side stream
            pass
        torch.cuda.current_stream(self.dev).wait_stream(sstream)
        if self.world == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(steps_per_graph):
                    pre()
                    post()
            self._graphs = (g, None)
        else:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                pre()
            with torch.cuda.graph(g2):
                post()
            self._graphs = (g1, g2)
        self._steps_per_graph = steps_per_graph
        torch.cuda.synchronize(self.dev)
        self.ctl.copy_(saved)

    def capture_group(self, k: int = 8):
        """World 1 with the folded update: also capture k consecutive resident steps as ONE HIP graph, so a run of
        steps pays one graph launch per k (replay_resident_n)."""
        if self.world != 1 or not getattr(self, "_fused", False) or k < 2:
            self._group = None
            return False
        torch.cuda.synchronize(self.dev)
        saved = self.ctl.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(k):
                if self._resident_fwd_bwd(self._stream()):
                    raise RuntimeError(_lib.lib().tgnx_last_error().decode())
        torch.cuda.synchronize(self.dev)
        self.ctl.copy_(saved)
        self._group = (k, g)
        return True

    def replay_resident_n(self, n: int):
        """n resident steps: whole k-step groups, then single replays (the same steps as n replay_resident calls)."""
        grp = getattr(self, "_group", None)
        done = 0
        while done < n:
            if grp and n - done >= grp[0]:
                grp[1].replay()
                done += grp[0]
            else:
                self.replay_resident()
                done += 1

    def replay_resident(self):
        """Run `steps_per_graph` resident steps from the captured graph(s)."""
        g1, g2 = self._graphs
        if g2 is None:
            g1.replay()
        else:
            g1.replay()
            self._allreduce_grads()
            g2.replay()

    def units(self):
        """(sum of assembled edges, sum of segments) since the last reset — roofline units."""
        return int(self.ctl[13]), int(self.ctl[14])

    # ------------------------------------------------------------------ status
    def check(self):
        err = int(self.ctl[CTL["ERR"]])
        if err:
            raise RuntimeError(f"tgnx TGNN step reported device error flags {err:#x} "
                               "(1: batch above capacity, 2: edge capacity exceeded)")

    def loss_sum(self) -> float:
        return float(self.ctl.view(torch.float64)[CTL["LOSS"]])

    def reset_loss(self):
        self.ctl.view(torch.float64)[CTL["LOSS"]] = 0.0

    def reset_counters(self):
        self.ctl[CTL["NB"]] = 0
