"""Drop-in `getModel` / `getOptimizer` (model_utils.py:700-710) backed by the fused HIP step.

`TGNN` mirrors the reference module tree so `state_dict()` keys are the
reference's (`temporal_encoder.w.weight`, `embedding_attn.edge_gatconv.fc_edge.weight`,
`predictor.src_fc.bias`, ...), but every trainable tensor is a view into one
flat fp32 buffer on the device, laid out by `tgnx_tgnn_param_layout`.  The
forward/backward/optimizer step run in libtgnx (tgnx/engine.py); there is no
torch-op path.

Initialisation follows the reference: TimeEncode w = 10^-linspace(0,9,D), b = 0
(model_utils.py:228-230); xavier_normal(gain=relu) on fc_node/fc_edge weights and
attn_{l,r,e} (:550-558); nn.Linear defaults for the biases and the predictor
(:176-184); memory = ones, requires_grad False (:267-271).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib

PARAM_ORDER = [  # flat-buffer order = tgnx_tgnn_param_layout
    "temporal_encoder.w.weight", "temporal_encoder.w.bias",
    "embedding_attn.edge_gatconv.attn_l", "embedding_attn.edge_gatconv.attn_r", "embedding_attn.edge_gatconv.attn_e",
    "embedding_attn.edge_gatconv.fc_node.weight", "embedding_attn.edge_gatconv.fc_node.bias",
    "embedding_attn.edge_gatconv.fc_edge.weight", "embedding_attn.edge_gatconv.fc_edge.bias",
    "predictor.src_fc.weight", "predictor.src_fc.bias", "predictor.dst_fc.weight", "predictor.dst_fc.bias",
    "predictor.out_fc.weight", "predictor.out_fc.bias",
]


class TgnnConfig(ctypes.Structure):
    _fields_ = [("num_nodes", ctypes.c_int64), ("ring", ctypes.c_int32), ("mem_dim", ctypes.c_int32),
                ("msg_dim", ctypes.c_int32), ("heads", ctypes.c_int32), ("max_batch", ctypes.c_int32),
                ("max_neg", ctypes.c_int32), ("feat_drop", ctypes.c_float), ("attn_drop", ctypes.c_float),
                ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float)]


def param_shapes(D: int, d: int, H: int) -> dict:
    F = d + D
    return {
        "temporal_encoder.w.weight": (D, 1), "temporal_encoder.w.bias": (D,),
        "embedding_attn.edge_gatconv.attn_l": (1, H, D), "embedding_attn.edge_gatconv.attn_r": (1, H, D),
        "embedding_attn.edge_gatconv.attn_e": (1, H, D),
        "embedding_attn.edge_gatconv.fc_node.weight": (H * D, D), "embedding_attn.edge_gatconv.fc_node.bias": (H * D,),
        "embedding_attn.edge_gatconv.fc_edge.weight": (H * D, F), "embedding_attn.edge_gatconv.fc_edge.bias": (H * D,),
        "predictor.src_fc.weight": (D, D), "predictor.src_fc.bias": (D,),
        "predictor.dst_fc.weight": (D, D), "predictor.dst_fc.bias": (D,),
        "predictor.out_fc.weight": (1, D), "predictor.out_fc.bias": (1,),
    }


def param_layout(cfg: TgnnConfig) -> list[int]:
    off = (ctypes.c_int64 * 16)()
    _lib.call("tgnx_tgnn_param_layout", ctypes.byref(cfg), off)
    return list(off)


def reference_init(D: int, d: int, H: int, generator: torch.Generator | None = None) -> dict:
    """CPU tensors with the reference's initialisation (see module docstring)."""
    g = generator
    gain = nn.init.calculate_gain("relu")
    out = {}

    def xavier(shape, fan_in, fan_out):
        std = gain * math.sqrt(2.0 / float(fan_in + fan_out))
        return torch.randn(shape, generator=g) * std

    def lin_bias(n, fan_in):
        bound = 1.0 / math.sqrt(fan_in)
        return (torch.rand(n, generator=g) * 2 - 1) * bound

    def lin_weight(o, i):  # kaiming_uniform(a=sqrt(5)) == U(-1/sqrt(i), 1/sqrt(i))
        bound = 1.0 / math.sqrt(i)
        return (torch.rand(o, i, generator=g) * 2 - 1) * bound

    F = d + D
    out["temporal_encoder.w.weight"] = torch.from_numpy(1 / 10 ** np.linspace(0, 9, D)).float().reshape(D, 1)
    out["temporal_encoder.w.bias"] = torch.zeros(D)
    # xavier fans of a [1,H,D] parameter as torch computes them: fan_in = H*D, fan_out = 1*D
    for k in ("attn_l", "attn_r", "attn_e"):
        out[f"embedding_attn.edge_gatconv.{k}"] = xavier((1, H, D), H * D, D)
    out["embedding_attn.edge_gatconv.fc_node.weight"] = xavier((H * D, D), D, H * D)
    out["embedding_attn.edge_gatconv.fc_node.bias"] = lin_bias(H * D, D)
    out["embedding_attn.edge_gatconv.fc_edge.weight"] = xavier((H * D, F), F, H * D)
    out["embedding_attn.edge_gatconv.fc_edge.bias"] = lin_bias(H * D, F)
    for k in ("src_fc", "dst_fc"):
        out[f"predictor.{k}.weight"] = lin_weight(D, D)
        out[f"predictor.{k}.bias"] = lin_bias(D, D)
    out["predictor.out_fc.weight"] = lin_weight(1, D)
    out["predictor.out_fc.bias"] = lin_bias(1, D)
    return out


class _Holder(nn.Module):
    pass


class TGNN(nn.Module):
    """Parameter container of the running reference model (model_utils.py:14-49)."""

    def __init__(self, ef_dim, hidden_dim, num_nodes, device, num_heads=8, layers=1, time_dim=100,
                 ring=10, max_batch=2048, max_neg=1, feat_drop=0.6, attn_drop=0.6, generator=None):
        super().__init__()
        dev = _lib.require_device(device)
        D, d, H = int(hidden_dim), int(ef_dim), int(num_heads)
        self.memory_dim = self.embedding_dim = D
        self.edge_feat_dim, self.num_heads, self.layers, self.num_nodes = d, H, layers, int(num_nodes)
        self.cfg = TgnnConfig(num_nodes=num_nodes, ring=ring, mem_dim=D, msg_dim=d, heads=H, max_batch=max_batch,
                              max_neg=max_neg, feat_drop=feat_drop, attn_drop=attn_drop, lr=1e-4, beta1=0.9,
                              beta2=0.999, eps=1e-8)
        self.offsets = param_layout(self.cfg)
        total = self.offsets[-1]
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad_flat = torch.zeros(total + 1, dtype=torch.float32, device=dev)   # + batch-loss slot
        self.time_assoc = torch.zeros(num_nodes, dtype=torch.float32, device=dev)   # model_utils.py:22
        shapes = param_shapes(D, d, H)
        init = reference_init(D, d, H, generator)
        # module tree with the reference's names
        self.memory = _Holder()
        self.memory.last_update_t = nn.Parameter(torch.zeros(num_nodes, device=dev), requires_grad=False)
        self.memory.memory = nn.Parameter(torch.ones(num_nodes, D, device=dev), requires_grad=False)
        self.temporal_encoder = _Holder()
        self.temporal_encoder.w = _Holder()
        self.embedding_attn = _Holder()
        self.embedding_attn.edge_gatconv = _Holder()
        self.embedding_attn.edge_gatconv.fc_node = _Holder()
        self.embedding_attn.edge_gatconv.fc_edge = _Holder()
        self.predictor = _Holder()
        for k in ("src_fc", "dst_fc", "out_fc"):
            setattr(self.predictor, k, _Holder())
        self._views = {}
        for name, off in zip(PARAM_ORDER, self.offsets[:-1]):
            n = int(np.prod(shapes[name]))
            view = self.flat[off:off + n].view(shapes[name])
            view.copy_(init[name].to(dev))
            p = nn.Parameter(view)
            mod = self
            parts = name.split(".")
            for part in parts[:-1]:
                mod = getattr(mod, part)
            setattr(mod, parts[-1], p)
            self._views[name] = (off, n, shapes[name])
        # the reference also reaches the encoder through embedding_attn (model_utils.py:34-36, 659)
        self.embedding_attn.temporal_encoder = self.temporal_encoder

    @property
    def device(self):
        return self.flat.device

    def trainable_count(self) -> int:
        return sum(n for _, n, _ in self._views.values())

    def load_reference_state(self, sd: dict) -> None:
        """Copy a reference-named state dict (e.g. an oracle or a reference checkpoint) into the flat buffer."""
        with torch.no_grad():
            for name, (off, n, shape) in self._views.items():
                self.flat[off:off + n].copy_(sd[name].reshape(-1).to(self.flat.device))
            if "memory.memory" in sd:
                self.memory.memory.copy_(sd["memory.memory"].to(self.flat.device))

    def grads_by_name(self) -> dict:
        return {name: self.grad_flat[off:off + n].view(shape) for name, (off, n, shape) in self._views.items()}

    def expose_grads(self) -> None:
        """Point each Parameter's .grad at its slice of the flat gradient buffer."""
        for name, (off, n, shape) in self._views.items():
            mod = self
            parts = name.split(".")
            for part in parts[:-1]:
                mod = getattr(mod, part)
            getattr(mod, parts[-1]).grad = self.grad_flat[off:off + n].view(shape)

    def forward(self, *args, **kwargs):
        raise RuntimeError("tgnx.TGNN runs through tgnx.epoch.train/test (the fused HIP step); the reference's "
                           "forward(g, ef, bt, blocks) takes a DGL graph, which this build replaces")


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (model_utils.py:709-710), applied by the HIP step to the flat buffer."""

    def __init__(self, model: TGNN, lr: float):
        params = [p for p in model.parameters() if p.requires_grad]
        super().__init__(params, dict(lr=lr, betas=(0.9, 0.999), eps=1e-8))
        self.model = model
        model.cfg.lr = float(lr)
        dev = model.flat.device
        self.exp_avg = torch.zeros_like(model.flat)
        self.exp_avg_sq = torch.zeros_like(model.flat)
        self._dev = dev

    def zero_grad(self, set_to_none: bool = True):
        pass  # the fused step overwrites the flat gradient buffer every batch

    def step(self, closure=None):
        raise RuntimeError("FusedAdam.step is applied inside tgnx.epoch.train (tgnx_tgnn_train_update)")


def getModel(feature_dim, hidden_dim, num_nodes, device, gnn_param=None, **kw):
    """model_utils.py:700-707.  When gnn_param came from tgnx's parse_config, the sampler width and the
    batch capacity default to the same file's sampling.neighbor[0] and train.batch_size."""
    from .data import config_of
    got = config_of(gnn_param) if gnn_param is not None else None
    if got is not None:
        if got[0].get("neighbor"):
            kw.setdefault("ring", int(got[0]["neighbor"][0]))
        if "batch_size" in got[3]:
            kw.setdefault("max_batch", int(got[3]["batch_size"]))
    if gnn_param is not None:
        gnn = TGNN(feature_dim, gnn_param["dim_out"], num_nodes, device, num_heads=gnn_param["att_head"],
                   layers=gnn_param["layer"], **kw)
    else:
        gnn = TGNN(feature_dim, hidden_dim, num_nodes, device, **kw)
    return {"gnn": gnn}


def getOptimizer(model, lr):
    return FusedAdam(model["gnn"], lr)
