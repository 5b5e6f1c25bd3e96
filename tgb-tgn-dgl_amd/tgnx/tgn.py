"""The TGN memory path (SURVEY §8 a14–a16) behind the reference's PyG surface.

`getModel` / `getOptimizer` mirror pyg_model_utils.py:10-43: the returned dict has 'memory' (TGNMemory:
time_enc + GRUCell, memory / last_update buffers, message stores), 'gnn' (GraphAttentionEmbedding:
TransformerConv, sharing memory.time_enc) and 'link_pred' (LinkPredictor); state_dict keys are the
reference's (`memory.memory_updater.weight_ih`, `gnn.conv.lin_key.weight`, `link_pred.lin_final.bias`, ...).  Every
trainable tensor is a view into one flat fp32 device buffer (`tgnx_tgn_param_layout`); the step runs in
libtgnx (TgnEngine below), there is no torch-op path.

Initialisation as the reference's modules: TimeEncoder = Linear(1, D) (torch default), GRUCell
U(-1/sqrt(D), 1/sqrt(D)), PyG Linear (kaiming_uniform a=sqrt(5) -> U(-1/sqrt(in), 1/sqrt(in)), bias the
same bound), LinkPredictor torch Linear defaults; memory / last_update zero (memory_module.py:106-110).
"""
from __future__ import annotations

import ctypes
import os
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib

P = ctypes.c_void_p

PARAM_ORDER = [  # flat-buffer order = tgnx_tgn_param_layout
    "memory.time_enc.lin.weight", "memory.time_enc.lin.bias",
    "memory.memory_updater.weight_ih", "memory.memory_updater.weight_hh", "memory.memory_updater.bias_ih",
    "memory.memory_updater.bias_hh",
    "gnn.conv.lin_key.weight", "gnn.conv.lin_key.bias", "gnn.conv.lin_query.weight", "gnn.conv.lin_query.bias",
    "gnn.conv.lin_value.weight", "gnn.conv.lin_value.bias", "gnn.conv.lin_edge.weight",
    "gnn.conv.lin_skip.weight", "gnn.conv.lin_skip.bias",
    "link_pred.lin_src.weight", "link_pred.lin_src.bias", "link_pred.lin_dst.weight", "link_pred.lin_dst.bias",
    "link_pred.lin_final.weight", "link_pred.lin_final.bias",
]
# layers = 2 (2-hop temporal attention, SURVEY §8d comment config): gnn.conv2 after the 21 above
PARAM_ORDER2 = PARAM_ORDER + [
    "gnn.conv2.lin_key.weight", "gnn.conv2.lin_key.bias", "gnn.conv2.lin_query.weight", "gnn.conv2.lin_query.bias",
    "gnn.conv2.lin_value.weight", "gnn.conv2.lin_value.bias", "gnn.conv2.lin_edge.weight",
    "gnn.conv2.lin_skip.weight", "gnn.conv2.lin_skip.bias",
]


class TgnConfig(ctypes.Structure):
    _fields_ = [("num_nodes", ctypes.c_int64), ("num_events", ctypes.c_int64), ("ring", ctypes.c_int32),
                ("mem_dim", ctypes.c_int32), ("msg_dim", ctypes.c_int32), ("heads", ctypes.c_int32),
                ("max_batch", ctypes.c_int32), ("max_neg", ctypes.c_int32), ("aggr", ctypes.c_int32),
                ("dropout", ctypes.c_float), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("layers", ctypes.c_int32),
                ("updater", ctypes.c_int32), ("emb_in_msg", ctypes.c_int32)]


class TgnBuffers(ctypes.Structure):
    _fields_ = [("ev_src", P), ("ev_dst", P), ("ev_t", P), ("ev_msg", P), ("neg", P), ("dst_nodes", P),
                ("n_dst", ctypes.c_int64), ("nbr", P), ("eid", P), ("rt", P), ("assoc", P), ("memory", P),
                ("last_update", P), ("store", P), ("node_gen", P), ("params", P), ("grads", P), ("adam_m", P),
                ("adam_v", P), ("ctl", P), ("out_pos", P), ("out_neg", P), ("mrr", P), ("ws", P), ("xrows", P),
                ("xcap", ctypes.c_int64), ("out_ev", P), ("plan_table", P), ("flags", ctypes.c_int32)]


# the memory modules' updater cell: TGNMemory.memory_updater (memory_module.py:70-78, memory_updater_cell
# 'gru' | 'rnn') and DyRepMemory.memory_updater (:259-264, memory_updater_type) — the same state-dict names
MEMORY_TYPES = ("tgn", "dyrep")


def param_shapes(D: int, d: int, layers: int = 1, updater: str = "gru") -> dict:
    Q = 3 * D + d
    G3 = 1 if updater == "rnn" else 3     # RNNCell: [D, .]; GRUCell: [3D, .] (r, z, n)
    u = "memory.memory_updater"
    s = {"memory.time_enc.lin.weight": (D, 1), "memory.time_enc.lin.bias": (D,),
         f"{u}.weight_ih": (G3 * D, Q), f"{u}.weight_hh": (G3 * D, D),
         f"{u}.bias_ih": (G3 * D,), f"{u}.bias_hh": (G3 * D,),
         "gnn.conv.lin_edge.weight": (D, D + d),
         "link_pred.lin_src.weight": (D, D), "link_pred.lin_src.bias": (D,),
         "link_pred.lin_dst.weight": (D, D), "link_pred.lin_dst.bias": (D,),
         "link_pred.lin_final.weight": (1, D), "link_pred.lin_final.bias": (1,)}
    convs = ("conv", "conv2") if layers == 2 else ("conv",)
    for cv in convs:
        for k in ("key", "query", "value", "skip"):
            s[f"gnn.{cv}.lin_{k}.weight"] = (D, D)
            s[f"gnn.{cv}.lin_{k}.bias"] = (D,)
        s[f"gnn.{cv}.lin_edge.weight"] = (D, D + d)
    return s


def reference_init(D: int, d: int, generator=None, layers: int = 1, updater: str = "gru") -> dict:
    g = generator

    def unif(shape, bound):
        return (torch.rand(shape, generator=g) * 2 - 1) * bound

    out = {}
    for name, shape in param_shapes(D, d, layers, updater).items():
        if name.startswith("memory.time_enc"):
            bound = 1.0                                   # Linear(1, D): fan_in = 1
        elif name.startswith("memory.memory_updater"):
            bound = 1.0 / math.sqrt(D)                    # GRUCell / RNNCell.reset_parameters
        elif name.endswith("lin_edge.weight"):
            bound = 1.0 / math.sqrt(D + d)
        else:
            bound = 1.0 / math.sqrt(D)                    # fan_in D (conv / predictor linears)
        out[name] = unif(shape, bound)
    return out


class _Holder(nn.Module):
    pass


class TGNModel(nn.Module):
    """memory + gnn + link_pred of pyg_model_utils.py:10-36 over one flat parameter buffer.

    memory = "tgn": TGNMemory (modules/memory_module.py:25-215) with memory_updater_cell = updater,
    "gru" (GRUCell, the default) or "rnn" (RNNCell, :70-78);
    memory = "dyrep": DyRepMemory (modules/memory_module.py:218-421) with memory_updater_type = updater; its
    use_src_emb_in_msg / use_dst_emb_in_msg (:387-408) build update_state's messages with the batch's
    embeddings (the TransformerConv output of the same forward: train / eval) in place of the memory rows of
    endpoints in src ∪ dst (1-hop embedding, world 1).  Without them its update order, messages and
    state-dict names are TGNMemory's."""

    def __init__(self, num_nodes, num_events, msg_dim, hidden_dim, device, ring=10, max_batch=2048, max_neg=1,
                 aggr="last", dropout=0.1, generator=None, layers=1, memory="tgn", updater="gru",
                 use_src_emb_in_msg=False, use_dst_emb_in_msg=False):
        super().__init__()
        if memory not in MEMORY_TYPES:
            raise ValueError(f"memory must be 'tgn' or 'dyrep', got {memory!r}")
        if updater not in ("gru", "rnn"):
            raise ValueError(f"Memory updater can be either 'gru' or 'rnn' (memory_module.py:75-78), got {updater!r}")
        emb = (1 if use_src_emb_in_msg else 0) | (2 if use_dst_emb_in_msg else 0)
        if emb and memory != "dyrep":
            raise ValueError("use_src/dst_emb_in_msg are DyRepMemory options (memory='dyrep'; memory_module.py:242-245)")
        if emb and int(layers) != 1:
            raise NotImplementedError("DyRep embedding messages are built for the 1-hop embedding (layers = 1)")
        self.memory_type, self.updater = memory, updater
        dev = _lib.require_device(device)
        D, d = int(hidden_dim), int(msg_dim)
        num_events = max(int(num_events or 0), 1)
        self.num_nodes, self.num_events, self.D, self.d = int(num_nodes), num_events, D, d
        self.cfg = TgnConfig(num_nodes=num_nodes, num_events=num_events, ring=ring, mem_dim=D, msg_dim=d, heads=2,
                             max_batch=max_batch, max_neg=max_neg, aggr=0 if aggr == "last" else 1, dropout=dropout,
                             lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, layers=int(layers),
                             updater=1 if updater == "rnn" else 0, emb_in_msg=emb)
        if layers not in (1, 2):
            raise ValueError(f"layers must be 1 or 2, got {layers}")
        self.layers = int(layers)
        order = PARAM_ORDER2 if layers == 2 else PARAM_ORDER
        self.param_order = order
        off = (ctypes.c_int64 * (len(order) + 1))()
        _lib.call("tgnx_tgn_param_layout", ctypes.byref(self.cfg), off)
        self.offsets = list(off)
        total = self.offsets[-1]
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad_flat = torch.zeros(total + 1, dtype=torch.float32, device=dev)    # + batch-loss slot
        shapes = param_shapes(D, d, layers, updater)
        init = reference_init(D, d, generator, layers, updater)
        self.memory = _Holder()
        self.memory.time_enc = _Holder()
        self.memory.time_enc.lin = _Holder()
        self.memory.memory_updater = _Holder()
        self.gnn = _Holder()
        self.gnn.conv = _Holder()
        if layers == 2:
            self.gnn.conv2 = _Holder()
        for cv in (("conv", "conv2") if layers == 2 else ("conv",)):
            for k in ("key", "query", "value", "edge", "skip"):
                setattr(getattr(self.gnn, cv), f"lin_{k}", _Holder())
        self.link_pred = _Holder()
        for k in ("src", "dst", "final"):
            setattr(self.link_pred, f"lin_{k}", _Holder())
        self._views = {}
        for name, o in zip(order, self.offsets[:-1]):
            n = int(np.prod(shapes[name]))
            view = self.flat[o:o + n].view(shapes[name])
            view.copy_(init[name].to(dev))
            mod = self
            parts = name.split(".")
            for part in parts[:-1]:
                mod = getattr(mod, part)
            setattr(mod, parts[-1], nn.Parameter(view))
            self._views[name] = (o, n, shapes[name])
        self.gnn.time_enc = self.memory.time_enc                           # shared (pyg_model_utils.py:27)
        # TGNMemory buffers (memory_module.py:80-83) and the message stores
        self.memory.register_buffer("memory", torch.zeros(num_nodes, D, device=dev))
        self.memory.register_buffer("last_update", torch.zeros(num_nodes, dtype=torch.long, device=dev))
        self.store = None
        self.ensure_events(max(int(num_events or 0), 1))
        self.node_gen = torch.zeros(num_nodes, dtype=torch.int32, device=dev)

    def ensure_events(self, n: int) -> None:
        """Size the message-store arena for an event table of n rows (the reference's getModel does
        not know the stream length; the engine calls this when it binds the table)."""
        if self.store is not None and n <= self.cfg.num_events:
            return
        self.cfg.num_events = int(n)
        self.num_events = int(n)
        words = _lib.lib().tgnx_tgn_store_words(ctypes.byref(self.cfg))
        if words == 0:
            raise RuntimeError(f"tgnx_tgn_store_words: {_lib.lib().tgnx_last_error().decode()}")
        old = self.store
        self.store = torch.zeros(int(words), dtype=torch.long, device=self.flat.device)
        if old is not None:   # per-node {off, cnt} words first; arena offsets stay valid
            self.store[:old.numel()].copy_(old)

    @property
    def device(self):
        return self.flat.device

    def trainable_count(self) -> int:
        return sum(n for _, n, _ in self._views.values())

    def load_reference_state(self, sd: dict) -> None:
        with torch.no_grad():
            for name, (o, n, _) in self._views.items():
                self.flat[o:o + n].copy_(sd[name].reshape(-1).to(self.flat.device))

    def grads_by_name(self) -> dict:
        """The last step's gradient of every parameter tensor (views into grad_flat).  Raises while an engine runs
        this model's steps with keep_grads=False (bench.py, the drop-in train()): those fused steps do not store the
        gradient (TGNX_TGN_NO_GRAD_STORE), so grad_flat would hold a stale step's values."""
        if getattr(self, "_grads_stale", False):
            raise RuntimeError("grads_by_name: the bound TgnEngine runs with keep_grads=False (fused Adam without the "
                               "gradient store): set engine.keep_grads = True before binding to read gradients")
        return {name: self.grad_flat[o:o + n].view(s) for name, (o, n, s) in self._views.items()}

    def settle(self) -> None:
        """Apply a data-parallel engine's deferred exchange (TgnEngine.finish) so that memory, last_update,
        the parameters and the Adam moments are current.  state_dict() calls it; direct
        reads of model.flat / model.memory.* between data-parallel steps need it (or engine.finish())."""
        f = self._tgnx_finish() if getattr(self, "_tgnx_finish", None) is not None else None
        if f is not None:
            f()

    def state_dict(self, *a, **k):
        self.settle()
        return super().state_dict(*a, **k)

    def forward(self, *a, **k):
        raise RuntimeError("tgnx TGN runs through tgnx.tgn.TgnEngine / pyg_epoch_utils (the fused HIP step)")


class TgnAdam(torch.optim.Optimizer):
    """torch.optim.Adam over set(memory) | set(gnn) | set(link_pred) (pyg_model_utils.py:38-43); the
    update runs on the device (tgnx_tgn_train_update)."""

    def __init__(self, model: TGNModel, lr: float):
        super().__init__([p for p in model.parameters() if p.requires_grad], dict(lr=lr, betas=(0.9, 0.999), eps=1e-8))
        self.model = model
        model.cfg.lr = float(lr)
        self.exp_avg = torch.zeros_like(model.flat)
        self.exp_avg_sq = torch.zeros_like(model.flat)

    def zero_grad(self, set_to_none: bool = True):
        pass

    def step(self, closure=None):
        raise RuntimeError("TgnAdam.step runs inside the TGN train step (tgnx_tgn_train_update)")


def row_header(v: int, lu: int) -> list:
    """Header of an exchanged memory row (include/tgnx.h TGNX_TGN_ROW; written on the device by the
    update step): node, last_update bits 0-23 / 24-47 / 48-63, each a float holding an exact integer."""
    b = int(lu) & 0xFFFFFFFFFFFFFFFF
    return [float(v), float(b & 0xFFFFFF), float((b >> 24) & 0xFFFFFF), float(b >> 48)]


def row_decode(h) -> tuple:
    """(node, last_update) of an exchanged row header (node -1: unused slot)."""
    b = int(h[1]) | (int(h[2]) << 24) | (int(h[3]) << 48)
    return int(h[0]), b - (1 << 64) if b >= 1 << 63 else b


def _p(t):
    return 0 if t is None else t.data_ptr()


EXCHANGE_MODES = ("fused", "split")


def exchange_collectives(comm, G: int, rank: int, world: int, mode: str = "fused", async_op: bool = False):
    """The data-parallel step's exchange over comm = [G gradient floats | world row slots] (each rank's kernels
    wrote its own slot):
      fused — ONE all-reduce of the whole buffer: the gradient sum, and (the other slots holding zeros) the
              all-gather of the rows, bit-exact (TgnEngine.__init__);
      split — an all-reduce of the G gradient floats and an in-place all_gather_into_tensor of the row slots:
              two collectives, but the rows travel once instead of as W-times-padded zeros in a sum.
    Returns the work handles (async_op) or []."""
    import torch.distributed as dist
    if mode == "split":
        rows = comm[G:]
        n = rows.numel() // world
        w1 = dist.all_reduce(comm[:G], async_op=async_op)
        w2 = dist.all_gather_into_tensor(rows, rows[rank * n:(rank + 1) * n], async_op=async_op)
        return [w for w in (w1, w2) if w is not None]
    if mode != "fused":
        raise ValueError(f"exchange mode must be one of {EXCHANGE_MODES}, got {mode!r}")
    w = dist.all_reduce(comm, async_op=async_op)
    return [] if w is None else [w]


class TgnEngine:
    """Owns the workspace of one TGN model + one neighbour ring over a resident event table
    (src, dst, t, msg rows = e_id).

    Data parallel (world > 1) resident steps defer the exchanged memory rows and Adam of step k to the head of
    step k + 1 (tgnx_tgn_train_fwd_bwd_pp).  Between such steps memory, last_update, the parameters and the
    Adam moments are one apply behind: call finish() before reading them directly.  check(), loss_sum(),
    flush(), eval / reset / binding calls and model.state_dict() do so themselves (the gradient buffer is final
    once the step's exchange returned: the apply does not change it)."""

    def __init__(self, model: TGNModel, loader, events: dict, optimizer: TgnAdam | None = None,
                 dst_nodes=None, seed: int = 0, rank: int = 0, world: int = 1, data_parallel: bool | None = None):
        self.model, self.loader, self.opt = model, loader, optimizer
        self.dev = model.device
        import weakref
        model._tgnx_finish = weakref.WeakMethod(self.finish)   # model.settle(): the deferred apply, if any
        cfg = model.cfg
        if cfg.ring != loader.size:
            cfg.ring = loader.size
        self.cfg = cfg
        ev = {k: torch.as_tensor(v) for k, v in events.items()}
        model.ensure_events(int(ev["src"].numel()))
        self.src = ev["src"].to(self.dev, torch.long).contiguous()
        self.dst = ev["dst"].to(self.dev, torch.long).contiguous()
        self.t = ev["t"].to(self.dev, torch.float32).contiguous()
        self.msg = ev["msg"].to(self.dev, torch.float32).contiguous()
        if self.src.numel() > cfg.num_events:
            raise ValueError("event table larger than cfg.num_events")
        nb = _lib.lib().tgnx_tgn_ws_bytes(ctypes.byref(cfg))
        if nb == 0:
            raise RuntimeError(f"tgnx_tgn_ws_bytes: {_lib.lib().tgnx_last_error().decode()}")
        self.ws = torch.zeros(nb, dtype=torch.uint8, device=self.dev)
        self.ctl = torch.zeros(24, dtype=torch.int64, device=self.dev)   # TGNX_CTL_WORDS
        self.neg_train = torch.zeros(cfg.num_events, dtype=torch.long, device=self.dev)
        self.out_pos = torch.zeros(cfg.max_batch, dtype=torch.float32, device=self.dev)
        self.out_neg = torch.zeros(cfg.max_batch * max(cfg.max_neg, 1), dtype=torch.float32, device=self.dev)
        self.mrr = torch.zeros(cfg.max_batch, dtype=torch.float64, device=self.dev)
        self.out_ev = None    # optional per-event train-output log (tgnx_tgn_buffers.out_ev)
        # the bound split's plan table (tgnx_tgn_plan_table; resident parity-set steps read it), TGNX_PLAN_TABLE=0: off
        self.plan_table = None
        self.use_plan_table = os.environ.get("TGNX_PLAN_TABLE", "1") != "0"
        self.dst_nodes = None if dst_nodes is None else torch.as_tensor(dst_nodes).to(self.dev, torch.long).contiguous()
        self.seed, self.rank, self.world = int(seed), int(rank), int(world)
        # the data-parallel step forms (exchange collective, then the apply + Adam launch): world > 1, or forced at
        # world 1 (data_parallel=True), where the exchange over a 1-rank group is an identity and the step must
        # equal the world-1 one (tests/test_gpu_tgn_rccl.py runs it through RCCL)
        self.dp = self.world > 1 if data_parallel is None else bool(data_parallel)
        if self.world > 1 and not self.dp:
            raise ValueError("TgnEngine: world > 1 needs the data-parallel step forms")
        self.fuse_adam = True
        # fused-Adam steps also store the gradient in model.grad_flat (grads_by_name); loops that never read it
        # (bench.py, the drop-in train()) set False before bind_resident: TGNX_TGN_NO_GRAD_STORE, 1.1 MB of
        # stores less per wiki-shaped step.  Data-parallel steps always write it (it is the exchange).
        self.keep_grads = True
        # resident steps fold the batch cursor into the step's first launch: tgnx_tgn_train_step_resident
        # (world 1, Adam fused) or tgnx_tgn_train_fwd_bwd_resident (world > 1; exchange + update follow).
        # Both forms are tested against advance + step per rank (test_gpu_tgn.py, test_gpu_tgn_dp.py).
        self.fold_cursor = True
        # resident steps pipeline across steps (world 1: tgnx_tgn_train_step_pipelined; world > 1:
        # tgnx_tgn_train_fwd_bwd_pipelined, then the exchange and tgnx_tgn_apply_rows_update): each step marks
        # and scans the next batch, so the next step starts at the message aggregation.  `_prefetched` says
        # whether the last call on these buffers was such a step (any other call clears it).
        self.pipeline = True
        # world > 1 pipelined steps leave the next batch's scan out of fwd_bwd and run it while the exchange
        # is in flight (tgnx_tgn_train_fwd_bwd_split + tgnx_tgn_scan_next)
        self.split_scan = True
        # world-1 1-hop pipelined steps alternate two parities of the scan's per-batch outputs
        # (tgnx_tgn_train_step_pp): the next batch is scanned into the other set mid-step instead of in the
        # step's last launch; `_parity` = the set the next step reads (two captured graphs)
        self.parity_sets = os.environ.get("TGNX_PP", "1") != "0"   # (TGNX_PP=0: same-box A/B against the fold)
        self._parity = 0
        self._prefetched = False
        self._prefetch_version = None
        # data-parallel parity-set steps (tgnx_tgn_train_fwd_bwd_pp): the exchanged rows + Adam of step k run at
        # the head of step k + 1's graph; `_apply_pending` = the last step's exchange is not applied yet
        # (finish() applies it eagerly: before reading memory / parameters / the loss, and before any other call)
        self._apply_pending = False
        if optimizer is None:
            self.adam_m, self.adam_v = torch.zeros_like(model.flat), torch.zeros_like(model.flat)
        else:
            self.adam_m, self.adam_v = optimizer.exp_avg, optimizer.exp_avg_sq
        # data parallel: each rank's GRU-updated memory rows [node | last_update | memory]
        # travel with the gradients in ONE all-reduce over RCCL: the exchange buffer is [gradients |
        # world x xcap rows]; a rank writes only its own row slot (exact small-integer floats, the
        # other slots zero), so the sum of the row part is the all-gather.  tgnx_tgn_apply_rows writes
        # them into memory / last_update on every rank and zeroes the slots for the next step.
        self.xrows = self.xgather = self.comm = None
        # the exchange collective: torch.distributed.all_reduce over the default group, unless a callable
        # (comm, async_op) -> work | None is set here (tools/dp_compute.py: a stand-in without a collective)
        self.exchange = None
        # fused: one all-reduce of [gradients | row slots]; split: gradient all-reduce + row all-gather
        # (exchange_collectives; TGNX_EXCHANGE, for the first 8-GPU A/B of the two)
        self.exchange_mode = os.environ.get("TGNX_EXCHANGE", "fused")
        if self.exchange_mode not in EXCHANGE_MODES:
            raise ValueError(f"TGNX_EXCHANGE must be one of {EXCHANGE_MODES}, got {self.exchange_mode!r}")
        if self.dp:
            self.xcap = min(cfg.num_nodes, 2 * (-(-cfg.max_batch // self.world)))
            rw = cfg.mem_dim + 4
            G = model.grad_flat.numel()
            self.comm = torch.zeros(G + self.world * self.xcap * rw, dtype=torch.float32, device=self.dev)
            self.comm[:G].copy_(model.grad_flat)
            model.grad_flat = self.comm[:G]          # the kernels' gradient buffer heads the exchange buffer
            self.xgather = self.comm[G:].view(self.world * self.xcap, rw)
            self.xrows = self.xgather[self.rank * self.xcap:(self.rank + 1) * self.xcap]

    def ensure_neg(self, kn: int) -> None:
        """Grow the workspace for eval batches with kn negatives per event (TGB: ~999 on tgbl-wiki)."""
        if kn <= self.cfg.max_neg:
            return
        torch.cuda.synchronize(self.dev)
        self.cfg.max_neg = int(kn)
        nb = _lib.lib().tgnx_tgn_ws_bytes(ctypes.byref(self.cfg))
        if nb == 0:
            raise RuntimeError(f"tgnx_tgn_ws_bytes: {_lib.lib().tgnx_last_error().decode()}")
        self.ws = torch.zeros(nb, dtype=torch.uint8, device=self.dev)   # scratch only: zero = initial state
        self.out_neg = torch.zeros(self.cfg.max_batch * kn, dtype=torch.float32, device=self.dev)
        self._prefetched = False
        if hasattr(self, "_res_buf"):
            self._res_buf = self._buffers(_p(self.neg_train))
            self._buf_ref = ctypes.byref(self._res_buf)
        self._graphs = None                                   # captured pointers are stale

    def _buffers(self, neg_ptr: int) -> TgnBuffers:
        m, ld = self.model, self.loader
        b = TgnBuffers()
        b.ev_src, b.ev_dst, b.ev_t, b.ev_msg = _p(self.src), _p(self.dst), _p(self.t), _p(self.msg)
        b.neg = neg_ptr
        b.dst_nodes = _p(self.dst_nodes)
        b.n_dst = 0 if self.dst_nodes is None else self.dst_nodes.numel()
        b.nbr, b.eid, b.rt, b.assoc = _p(ld.neighbors), _p(ld.e_id), _p(ld.t), _p(ld._assoc)
        b.memory, b.last_update = _p(m.memory.memory), _p(m.memory.last_update)
        b.store, b.node_gen = _p(m.store), _p(m.node_gen)
        b.params, b.grads, b.adam_m, b.adam_v = _p(m.flat), _p(m.grad_flat), _p(self.adam_m), _p(self.adam_v)
        b.ctl, b.out_pos, b.out_neg, b.mrr, b.ws = _p(self.ctl), _p(self.out_pos), _p(self.out_neg), _p(self.mrr), _p(self.ws)
        b.xrows, b.xcap = _p(self.xrows), (0 if self.xrows is None else self.xcap)
        b.out_ev = _p(self.out_ev)
        b.plan_table = _p(self.plan_table)
        b.flags = 0 if self.keep_grads else 1   # TGNX_TGN_NO_GRAD_STORE
        # steps on these buffers leave grad_flat stale (fused Adam without the store; data-parallel steps always
        # write it: it heads the exchange buffer)
        m._grads_stale = not self.keep_grads and not self.dp
        return b

    def _stream(self):
        return _lib.stream(self.dev)

    def advance(self, batch_start: int, B: int, train: bool):
        self.finish()
        self._prefetched = False
        _lib.call("tgnx_tgnn_advance", _p(self.ctl), 0, batch_start, B, batch_start, 0, 0, 1, self.rank, self.world,
                  self.seed, 1 if train else 0, self._stream())

    # ------------------------------------------------------------------ state
    def reset_state(self):
        """memory_module.reset_state + neighbor_loader.reset_state (pyg_epoch_utils.py:15-16)."""
        self.finish()
        self._prefetched = False
        b = self._buffers(0)
        _lib.call("tgnx_tgn_reset_state", ctypes.byref(self.cfg), ctypes.byref(b), self._stream())
        self.loader.reset_state()

    def flush(self):
        """TGNMemory.train(False) (memory_module.py:209-215)."""
        self.finish()
        self._prefetched = False
        b = self._buffers(0)
        nb = int(_lib.lib().tgnx_tgn_flush_scratch_bytes(ctypes.byref(self.cfg)))
        # graphs beyond one workspace chunk: a snapshot of memory / last_update.  It is allocated on, and
        # the flush runs on, the current stream, so the caching allocator reuses the block only for work
        # queued after the flush: it may go out of scope when this call returns
        scratch = torch.empty(max(nb, 16), dtype=torch.uint8, device=self.dev) if nb else None
        _lib.call("tgnx_tgn_flush", ctypes.byref(self.cfg), ctypes.byref(b), _p(scratch), nb, self._stream())

    # ------------------------------------------------------------------ steps
    def train_batch(self, start: int, B: int, neg=None, dropout: bool = True, update: bool = True):
        """One TGN train batch over events [start, start + B).  neg: LongTensor[B] to inject, or None to
        draw on the device.  Returns (sigmoid(pos), sigmoid(neg)) views."""
        if neg is not None:
            self.neg_train[start:start + B].copy_(torch.as_tensor(neg).to(self.dev, torch.long))
        self.advance(start, B, True)
        b = self._buffers(_p(self.neg_train))
        fused = update and self._fused()
        _lib.call("tgnx_tgn_train_step" if fused else "tgnx_tgn_train_fwd_bwd", ctypes.byref(self.cfg), ctypes.byref(b),
                  0 if neg is not None else 1, 1 if dropout else 0, self._stream())
        self._pending = b
        if update and not fused:
            self.apply_update()
        return self.out_pos[:B], self.out_neg[:B]

    def _fused(self) -> bool:
        """Adam folded into the step's gradient writers (tgnx_tgn_train_step): world 1 only, since data
        parallel steps all-reduce the gradients before the update."""
        return self.fuse_adam and not self.dp

    def apply_update(self, allreduce: bool = True):
        if allreduce and self.dp:
            self._exchange()
        if self.dp:   # the exchanged rows and Adam in one launch
            _lib.call("tgnx_tgn_apply_rows_update", ctypes.byref(self.cfg), ctypes.byref(self._pending),
                      _p(self.xgather), self.xgather.shape[0], self._stream())
        else:
            _lib.call("tgnx_tgn_train_update", ctypes.byref(self.cfg), ctypes.byref(self._pending), self._stream())

    def _exchange(self):
        """The step's one collective: gradient sum and the touched memory rows of every rank (an
        all-gather carried by the same all-reduce, see __init__)."""
        if self.exchange is not None:
            self.exchange(self.comm, False)
            return
        exchange_collectives(self.comm, self.model.grad_flat.numel(), self.rank, self.world, self.exchange_mode)

    def _apply_rows(self, b):
        _lib.call("tgnx_tgn_apply_rows", ctypes.byref(self.cfg), ctypes.byref(b), _p(self.xgather),
                  self.xgather.shape[0], self._stream())

    def eval_batch(self, start: int, B: int, negs):
        """TGB-style eval batch: negs LongTensor[B, Kn].  Returns (pos [B], neg [B, Kn], rr [B])."""
        negs = torch.as_tensor(negs).to(self.dev, torch.long).contiguous()
        Kn = negs.shape[1]
        self.ensure_neg(Kn)
        self.advance(start, B, False)
        # the kernels index neg[(start + i) * Kn + c]: shift the base pointer by start rows
        b = self._buffers(negs.data_ptr() - start * Kn * 8)
        _lib.call("tgnx_tgn_eval_step", ctypes.byref(self.cfg), ctypes.byref(b), Kn, self._stream())
        self._keep = negs
        return self.out_pos[:B], self.out_neg[:B * Kn].view(B, Kn), self.mrr[:B]

    # ------------------------------------------------------------------ resident (graph-capturable)
    def bind_resident(self, split_lo: int, split_hi: int, batch: int, dropout: bool = True):
        """Consecutive batches of `batch` events over [split_lo, split_hi), negatives drawn on the
        device; the batch cursor lives in the control block (no host arguments change per step)."""
        self.finish()
        self._group = None   # (a step group captured for a previous binding)
        self._res = (int(split_lo), int(split_hi), int(batch))
        self._res_drop = 1 if dropout else 0
        self._prefetched = False
        self._release_plan_table()
        if self.use_plan_table:   # the split's ring-insert / store plans, built once for every batch
            nbytes = int(_lib.lib().tgnx_tgn_plan_table_bytes(ctypes.byref(self.cfg), *self._res))
            if nbytes == 0:
                raise RuntimeError(f"tgnx_tgn_plan_table_bytes: {_lib.lib().tgnx_last_error().decode()}")
            self.plan_table = torch.empty(nbytes, dtype=torch.uint8, device=self.dev)
            _lib.call("tgnx_tgn_plan_table", ctypes.byref(self.cfg), ctypes.byref(self._buffers(0)), *self._res,
                      _p(self.plan_table), nbytes, self._stream())
        self._res_buf = self._buffers(_p(self.neg_train))
        L = _lib.lib()
        self._res_fused = self._fused()
        self._f = (L.tgnx_tgnn_advance, L.tgnx_tgn_train_step if self._res_fused else L.tgnx_tgn_train_fwd_bwd,
                   L.tgnx_tgn_train_update, L.tgnx_tgn_apply_rows_update)
        self._cfg_ref, self._buf_ref = ctypes.byref(self.cfg), ctypes.byref(self._res_buf)
        self._ctl_p = ctypes.c_void_p(self.ctl.data_ptr())

    def _release_plan_table(self):
        """Drop the bound split's plan table, and the library's record of it (tgnx_tgn_plan_table_release): the
        caching allocator may hand its address to another tensor."""
        if self.plan_table is not None and hasattr(_lib.lib(), "tgnx_tgn_plan_table_release"):
            torch.cuda.synchronize(self.dev)      # (no step still reading it)
            _lib.lib().tgnx_tgn_plan_table_release(ctypes.c_void_p(self.plan_table.data_ptr()))
        self.plan_table = None

    def __del__(self):
        try:
            if getattr(self, "plan_table", None) is not None:
                _lib.lib().tgnx_tgn_plan_table_release(ctypes.c_void_p(self.plan_table.data_ptr()))
        except Exception:
            pass

    def begin_epoch(self):
        """pyg_epoch_utils.py:11-16: memory reset_state + neighbor_loader reset_state; cursor to 0."""
        self.reset_state()
        self.ctl[10] = 0
        self._prefetched = False

    def _pipelined(self) -> bool:
        return self.pipeline and self.fold_cursor and (self._res_fused or self.dp)

    def _pp(self) -> bool:
        """Parity-set steps: world 1 with Adam fused (tgnx_tgn_train_step_pp), or data parallel
        (tgnx_tgn_train_fwd_bwd_pp: the previous step's exchanged rows + Adam at the head of the step); 1 or 2
        hops (TGNX_PP_2HOP=0 keeps 2 hops on the pipelined step: comment-shaped 0.2462 vs 0.2383 ms)."""
        if not (self.parity_sets and self._pipelined()):
            return False
        if self.model.layers == 2 and os.environ.get("TGNX_PP_2HOP", "1") == "0":
            return False
        return self._res_fused if not self.dp else True

    def _dp_pp(self) -> bool:
        return self.dp and self._pp()

    def _pre(self, prefetched: bool = False, parity=None, apply=None):
        adv, fb = self._f[:2]
        lo, hi, batch = self._res
        st = self._stream()
        par = self._parity if parity is None else parity
        if self._dp_pp():
            ap = self._apply_pending if apply is None else apply
            rc = _lib.lib().tgnx_tgn_train_fwd_bwd_pp(self._cfg_ref, self._buf_ref, lo, hi, batch, self.rank, self.world,
                                                     self.seed, self._res_drop, 1 if prefetched else 0, par,
                                                     1 if ap else 0, ctypes.c_void_p(self.xgather.data_ptr()),
                                                     ctypes.c_int64(self.xgather.shape[0]), st)
        elif self._pp():
            rc = _lib.lib().tgnx_tgn_train_step_pp(self._cfg_ref, self._buf_ref, lo, hi, batch, self.seed, self._res_drop,
                                                  1 if prefetched else 0, par, st)
        elif self._pipelined() and self._res_fused:
            rc = _lib.lib().tgnx_tgn_train_step_pipelined(self._cfg_ref, self._buf_ref, lo, hi, batch, self.seed,
                                                         self._res_drop, 1 if prefetched else 0, st)
        elif self._pipelined():
            f = _lib.lib().tgnx_tgn_train_fwd_bwd_split if self._split() else _lib.lib().tgnx_tgn_train_fwd_bwd_pipelined
            rc = f(self._cfg_ref, self._buf_ref, lo, hi, batch, self.rank, self.world, self.seed, self._res_drop,
                   1 if prefetched else 0, st)
        elif self.fold_cursor:   # the batch cursor folded into the step's first launches
            f = _lib.lib().tgnx_tgn_train_step_resident if self._res_fused else _lib.lib().tgnx_tgn_train_fwd_bwd_resident
            rc = f(self._cfg_ref, self._buf_ref, lo, hi, batch, self.rank, self.world, self.seed, self._res_drop, st)
        else:
            rc = adv(self._ctl_p, 1, 0, 0, 0, lo, hi, batch, self.rank, self.world, self.seed, 1, st)
            rc |= fb(self._cfg_ref, self._buf_ref, 1, self._res_drop, st)
        if rc:
            raise RuntimeError(f"tgnx TGN resident step failed: {_lib.lib().tgnx_last_error().decode()}")

    def _post(self):
        st = self._stream()
        rc = 0
        if self.dp:   # the exchanged rows and Adam, one launch
            rc |= self._f[3](self._cfg_ref, self._buf_ref, ctypes.c_void_p(self.xgather.data_ptr()),
                             ctypes.c_int64(self.xgather.shape[0]), st)
        elif not self._res_fused:   # fused step: Adam already applied
            rc |= self._f[2](self._cfg_ref, self._buf_ref, st)
        if rc:
            raise RuntimeError(f"tgnx TGN resident update failed: {_lib.lib().tgnx_last_error().decode()}")

    def _split(self) -> bool:
        return self.split_scan and self.dp and self._pipelined() and not self._res_fused and not self._pp()

    def _scan_next(self):
        """The next batch's scan (split pipelined steps): rides beside the exchange."""
        if self._split():
            lo, hi, batch = self._res
            rc = _lib.lib().tgnx_tgn_scan_next(self._cfg_ref, self._buf_ref, lo, hi, batch, self.rank, self.world,
                                               self.seed, self._stream())
            if rc:
                raise RuntimeError(f"tgnx_tgn_scan_next failed: {_lib.lib().tgnx_last_error().decode()}")

    def _allreduce(self, between=None):
        """The exchange; `between` (the next batch's scan) runs on the compute stream while it is in flight."""
        if self.dp:
            if self.exchange is not None:
                work = self.exchange(self.comm, True)
                works = [] if work is None else [work]
            else:
                works = exchange_collectives(self.comm, self.model.grad_flat.numel(), self.rank, self.world,
                                             self.exchange_mode, async_op=True)
            if between is not None:
                between()
            for w in works:
                w.wait()
        elif between is not None:
            between()

    def _prefetch_valid(self) -> bool:
        """The previous pipelined step's preparation of this batch still holds: no other engine call since
        (tracked by _prefetched) and no host-side change of the ring through the loader (its version)."""
        return self._prefetched and getattr(self.loader, "version", None) == self._prefetch_version

    def _mark_prefetched(self):
        self._prefetched = self._pipelined()
        self._prefetch_version = getattr(self.loader, "version", None)

    def resident_train_step(self):
        if self._dp_pp():   # [apply(k - 1) ‖ step k], then the exchange; its apply heads the next step
            self._pre(self._prefetch_valid(), apply=self._apply_pending)
            self._apply_pending = False
            self._allreduce()
            self._apply_pending = True
            self._mark_prefetched()
            self._parity ^= 1
            return
        self._pre(self._prefetch_valid())
        self._allreduce(self._scan_next)
        self._post()
        self._mark_prefetched()
        self._parity ^= 1 if self._pp() else 0

    def finish(self):
        """Apply a data-parallel parity-set step's exchange now (tgnx_tgn_apply_rows_update: the gathered
        memory rows and Adam) instead of at the head of the next step.  Every call that reads or rewrites the
        state runs this first; replays then take the graph without the apply."""
        if not self._apply_pending:
            return
        rc = _lib.lib().tgnx_tgn_apply_rows_update(self._cfg_ref, self._buf_ref, ctypes.c_void_p(self.xgather.data_ptr()),
                                                  ctypes.c_int64(self.xgather.shape[0]), self._stream())
        self._apply_pending = False
        if rc:
            raise RuntimeError(f"tgnx_tgn_apply_rows_update failed: {_lib.lib().tgnx_last_error().decode()}")

    def capture_resident(self):
        """One resident step as HIP graph(s) (world > 1: the collectives stay eager between them)."""
        torch.cuda.synchronize(self.dev)
        saved = self.ctl.clone()
        if self._dp_pp():   # per parity, with and without the previous step's apply at its head; the collective stays eager
            gd = {}
            for par in (0, 1):
                for ap in (0, 1):
                    gd[par, ap] = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gd[par, ap]):
                        self._pre(True, par, bool(ap))
            self._graphs = (gd, None, None)
        elif not self.dp and self._pp():   # one graph per parity, replayed alternately
            gp = (torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph())
            for par in (0, 1):
                with torch.cuda.graph(gp[par]):
                    self._pre(True, par)
            self._graphs = (gp, None, None)
        elif not self.dp:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):   # pipelined: the steady-state step (the previous step prefetched)
                self._pre(True)
                self._post()
            self._graphs = (g, None, None)
        else:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):   # pipelined: the steady-state step (the previous step prefetched)
                self._pre(self._pipelined())
            gs = None
            if self._split():
                gs = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gs):
                    self._scan_next()
            with torch.cuda.graph(g2):
                self._post()
            self._graphs = (g1, g2, gs)
        torch.cuda.synchronize(self.dev)
        self.ctl.copy_(saved)

    def capture_group(self, k: int = 8):
        """World 1, parity-set steps: also capture k consecutive steps (parities 0, 1, 0, ...) as ONE HIP graph, so a
        run of steps pays one graph launch per k (replay_resident_n).  k even: the group starts and ends at parity 0."""
        if self.dp or not self._pp() or k < 2 or k % 2:
            self._group = None
            return False
        torch.cuda.synchronize(self.dev)
        saved = self.ctl.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for q in range(k):
                self._pre(True, q & 1)
        torch.cuda.synchronize(self.dev)
        self.ctl.copy_(saved)
        self._group = (k, g)
        return True

    def replay_resident_n(self, n: int):
        """n resident steps: whole captured k-step groups wherever the set parity and the prefetch allow, single
        replays (or the priming eager step) otherwise.  The same steps as n calls of replay_resident()."""
        grp = getattr(self, "_group", None)
        done = 0
        while done < n:
            if grp and n - done >= grp[0] and self._parity == 0 and self._prefetch_valid():
                grp[1].replay()
                self._mark_prefetched()
                done += grp[0]
            else:
                self.replay_resident()
                done += 1

    def replay_resident(self):
        g1, g2, gs = self._graphs
        if self._pipelined() and not self._prefetch_valid():
            self.resident_train_step()   # marks + scans this batch first (eager), prefetches the next
            return
        if isinstance(g1, dict):   # data-parallel parity graphs
            g1[self._parity, 1 if self._apply_pending else 0].replay()
            self._apply_pending = False
            self._allreduce()
            self._apply_pending = True
            self._parity ^= 1
            self._mark_prefetched()
            return
        if isinstance(g1, tuple):   # parity graphs
            g1[self._parity].replay()
            self._parity ^= 1
            self._mark_prefetched()
            return
        g1.replay()
        if g2 is not None:
            self._allreduce(gs.replay if gs is not None else None)
            g2.replay()
        self._mark_prefetched()

    def units(self):
        """(sum of sampled edges, sum of sampled nodes) since the last reset."""
        return int(self.ctl[13]), int(self.ctl[14])

    def loss_sum(self) -> float:
        self.finish()   # (the loss sum is accumulated by the Adam launch)
        return float(self.ctl[12:13].view(torch.float64).item())

    ERR_BITS = {4: "batch or sampled node / edge set beyond the workspace capacity",
                8: "more updated memory rows than the exchange slots hold (xcap)",
                16: "stale scan-output set: tgnx_tgn_train_step_pp / _fwd_bwd_pp called with the wrong parity, "
                    "or a prefetch that no longer holds",
                32: "edge sort beyond its LDS counters"}

    def check(self, settle: bool = True):
        """Raise on the step error flags (ctl[11]).  settle: first apply a deferred data-parallel exchange
        (finish()), so the state is current afterwards; False leaves it pending (tests that perform the
        exchange themselves after the step returned)."""
        if settle:
            self.finish()
        err = int(self.ctl[11].item())
        if err:
            why = "; ".join(m for b, m in self.ERR_BITS.items() if err & b) or "unknown"
            raise RuntimeError(f"tgnx TGN step error flags {err:#x}: {why}")


# config/TGN.yml memory section -> the PyG TGN's modules (TGL key names; TGN.yml:10-18)
MAIL_COMBINE = {"last": "last", "mean": "mean"}          # msg_agg.py LastAggregator / MeanAggregator
MEMORY_UPDATE = {"gru": "gru", "rnn": "rnn"}             # memory_module.py:70-78 memory_updater_cell


def model_options(gnn_param=None, memory_param=None, sample_param=None, train_param=None) -> dict:
    """TGNModel keywords from config/TGN.yml sections (utils.parse_config order).  gnn: `layer` -> layers
    (attention hops, 1 or 2); memory: `mail_combine` -> aggr, `memory_update` -> updater, `type` must be
    'node' (TGL's 'none' is a memory-less model, not the TGN path); sampling: `neighbor[0]` -> ring;
    train: `batch_size` -> max_batch.  When only gnn_param is given and it came from tgnx's parse_config
    (as in pyg-mem-tgn.py:36,49), the other sections of the same file are used."""
    from .data import config_of
    if gnn_param is not None and memory_param is None:
        got = config_of(gnn_param)
        if got is not None:
            sample_param = sample_param if sample_param is not None else got[0]
            memory_param = got[1]
            train_param = train_param if train_param is not None else got[3]
    out = {}
    if gnn_param is not None and "layer" in gnn_param:
        out["layers"] = int(gnn_param["layer"])
    if memory_param is not None:
        typ = memory_param.get("type", "node")
        if typ != "node":
            raise NotImplementedError(f"memory.type {typ!r}: only 'node' memory (TGNMemory) is the TGN path")
        mc = memory_param.get("mail_combine", "last")
        if mc not in MAIL_COMBINE:
            raise ValueError(f"memory.mail_combine must be 'last' or 'mean' (msg_agg.py), got {mc!r}")
        mu = memory_param.get("memory_update", "gru")
        if mu not in MEMORY_UPDATE:
            raise ValueError(f"memory.memory_update must be 'gru' or 'rnn' (memory_module.py:70-78), got {mu!r}")
        out["aggr"], out["updater"] = MAIL_COMBINE[mc], MEMORY_UPDATE[mu]
    if sample_param is not None and sample_param.get("neighbor"):
        out["ring"] = int(sample_param["neighbor"][0])
    if train_param is not None and "batch_size" in train_param:
        out["max_batch"] = int(train_param["batch_size"])
    return out


def getModel(feature_dim, hidden_dim, num_nodes, device, gnn_param=None, memory_param=None, num_events=None, **kw):
    """pyg_model_utils.py:10-36 with the call of pyg-mem-tgn.py:49 (`gnn_param=`; the reference's own
    getModel lacks it): hidden_dim is the memory / time / embedding width (gnn dim_out), and the config
    sections select the model (model_options: layer, mail_combine, memory_update, neighbor, batch_size).
    num_events (optional) pre-sizes the message-store arena; otherwise the engine sizes it when it binds
    the event table.  Explicit keywords win over the config: ring, max_batch, max_neg, aggr, dropout,
    layers, updater = 'gru' | 'rnn' (TGNMemory memory_updater_cell), memory = 'tgn' | 'dyrep'
    (DyRepMemory as the memory module, modules/memory_module.py:218-421; TGNModel)."""
    opts = model_options(gnn_param, memory_param)
    opts.update(kw)
    m = TGNModel(num_nodes, num_events, feature_dim, hidden_dim, device, **opts)
    return {"memory": m.memory, "gnn": m.gnn, "link_pred": m.link_pred, "model": m}


def getOptimizer(model, lr):
    return TgnAdam(model["model"], lr)
