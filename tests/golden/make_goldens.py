"""Capture golden vectors from the reference's own modules (run in the build container only).

    python tests/golden/make_goldens.py  [--ref /root/reference]

The reference is pure Python; the modules on the hot path that import without
DGL / PyG / TGB are executed here on small seeded synthetic
inputs and their outputs are written as `.npz` fixtures next to this script.
Nothing from the reference (source or bytecode) is copied; only numbers.

Modules exercised (file:line of the code that produced each fixture):
  sampler_*.npz  neighbor_loader.py:15-109   LastNeighborLoader call/insert/reset
  blocks.npz     dependencyGraph.py:8-49     get_block / dependecyAwareBatch
  negs.npz       neg_sampler.py:3-23         NegLinkSamplerDest.sample under torch.manual_seed
  dataset.npz    temporal_dataset.py:34-57   TemporalGraphDataset + default collate
  model.npz      model_utils.py:165-237,700  TimeEncode, EdgePredictor, TGNN parameter shapes
                 (model_utils imports `dgl` at module scope; a placeholder module that only
                 provides the imported names is put in sys.modules so the pure-torch classes
                 can be instantiated — no DGL op is ever called)
  msg.npz        modules/msg_func.py:12-18   IdentityMessage
  link_pred.npz  modules/decoder.py:12-27  LinkPredictor (sigmoid output)
  tgn_memory_*.npz  modules/memory_module.py:25-215 + msg_agg.py:15-26 + msg_func.py:12-18
                 TGNMemory itself (IdentityMessage, Last / MeanAggregator, GRUCell / RNNCell): train-mode
                 memory(n_id) and update_state over several batches, train(False) (the flush), eval-mode
                 memory(n_id) and update_state — every returned tensor and the memory / last_update
                 buffers after each call.  Its missing third-party imports get placeholder modules
                 (torch_geometric.nn.inits.zeros, torch_geometric.utils.scatter, torch_scatter.scatter_max,
                 modules.time_enc.TimeEncoder) that restate those functions' published behaviour; so the
                 fixture pins the module's own control flow — store layout and ordering, update-vs-store
                 order in train / eval, _compute_msg's t_rel, the flush — while the placeholder arithmetic
                 (scatter, the time encoder) stays parity-unpinned
  tgn_model_wiring.npz  pyg_model_utils.py:10-43 getModel / getOptimizer as written + emb_module.py:11-29 +
                 decoder.py LinkPredictor + neighbor_loader.py, driven by the canonical PyG TGN batch
                 (pyg_epoch_utils.py:106-137): outputs, loss, every parameter gradient, memory / last_update
                 per batch over 4 batches with Adam; a torch_geometric.nn.TransformerConv placeholder (PyG's
                 published semantics) added to the ones above — pins the wiring (rel_t sign, edge_attr order,
                 the shared time encoder, the composition), not the placeholders' arithmetic
"""
from __future__ import annotations

import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _collision_free_batches(rng, num_nodes, num_batches, batch, K):
    """Batches in which no node occurs more than K times among (src ∪ dst) entries.

    For such batches the reference's survivor set is deterministic (neighbor_loader.py:68
    sorts with an unstable sort; with <=K entries per node every entry survives the scatter).
    """
    out = []
    for _ in range(num_batches):
        cnt = np.zeros(num_nodes, dtype=np.int64)
        s, d = [], []
        while len(s) < batch:
            a, b = rng.integers(0, num_nodes, size=2)
            need = np.zeros(num_nodes, dtype=np.int64)
            need[a] += 1
            need[b] += 1
            if (cnt + need).max() > K:
                continue
            cnt += need
            s.append(a)
            d.append(b)
        out.append((np.array(s, dtype=np.int64), np.array(d, dtype=np.int64)))
    return out


def capture_sampler(ref, name, num_nodes, K, num_batches, batch, monotone, seed):
    from neighbor_loader import LastNeighborLoader
    rng = np.random.default_rng(seed)
    batches = _collision_free_batches(rng, num_nodes, num_batches, batch, K)
    loader = LastNeighborLoader(num_nodes, size=K, device="cpu")
    rec = {k: [] for k in ["q", "q_off", "nid", "nid_off", "ei", "eid", "et", "e_off",
                            "assoc_nid", "ins_src", "ins_dst", "ins_t", "ins_off",
                            "state_eid", "state_t", "state_nbr", "ins_assoc"]}
    t0 = 0.0
    q_off = nid_off = e_off = ins_off = 0
    for bi, (s, d) in enumerate(batches):
        # query: the batch endpoints plus some random nodes (sorted unique, like epoch_utils.py:215)
        extra = rng.integers(0, num_nodes, size=batch)
        q = np.unique(np.concatenate([s, d, extra]))
        n_id, ei, e_id, et = loader(torch.from_numpy(q))
        rec["q"].append(q); rec["q_off"].append(q_off); q_off += q.shape[0]
        rec["nid"].append(n_id.numpy()); rec["nid_off"].append(nid_off); nid_off += n_id.shape[0]
        rec["assoc_nid"].append(loader._assoc[n_id].numpy())
        rec["ei"].append(ei.numpy().T); rec["eid"].append(e_id.numpy()); rec["et"].append(et.numpy())
        rec["e_off"].append(e_off); e_off += e_id.shape[0]
        if monotone:
            tt = t0 + np.sort(rng.integers(0, 50, size=batch)).astype(np.float32)
            t0 = float(tt.max())
        else:
            tt = rng.integers(0, 10_000, size=batch).astype(np.float32)
        loader.insert(torch.from_numpy(s), torch.from_numpy(d), torch.from_numpy(tt))
        touched = np.unique(np.concatenate([s, d]))
        rec["ins_assoc"].append(loader._assoc[torch.from_numpy(touched)].numpy())
        rec["ins_src"].append(s); rec["ins_dst"].append(d); rec["ins_t"].append(tt)
        rec["ins_off"].append(ins_off); ins_off += batch
        eid = loader.e_id.numpy().copy()
        nbr = loader.neighbors.numpy().copy()
        nbr[eid < 0] = -1           # neighbours of empty slots are uninitialised memory
        rec["state_eid"].append(eid); rec["state_t"].append(loader.t.numpy().copy())
        rec["state_nbr"].append(nbr)
    out = {}
    for k, v in rec.items():
        if k.endswith("_off"):
            out[k] = np.array(v + [None], dtype=object)[:-1].astype(np.int64)
        elif k.startswith("state"):
            out[k] = np.stack(v)
        else:
            out[k] = np.concatenate(v)
    out["meta"] = np.array([num_nodes, K, num_batches, batch, int(monotone)], dtype=np.int64)
    # reset_state (neighbor_loader.py:106-109)
    loader.reset_state()
    out["reset_eid_min"] = np.array([loader.e_id.min().item(), loader.e_id.max().item(), loader.cur_e_id])
    np.savez_compressed(os.path.join(HERE, f"sampler_{name}.npz"), **out)


def capture_blocks(seed):
    from dependencyGraph import get_block, dependecyAwareBatch
    from temporal_dataset import TemporalGraphDataset
    from torch.utils.data import DataLoader
    rng = np.random.default_rng(seed)
    # Zipf-ish small stream so blocks get deep
    E, N, B = 1500, 60, 200
    p = np.arange(1, N + 1, dtype=np.float64) ** -1.3
    p /= p.sum()
    src = rng.choice(N, size=E, p=p).astype(np.int64)
    dst = rng.choice(N, size=E, p=p[::-1] / p.sum()).astype(np.int64)
    t = np.sort(rng.integers(0, 1000, size=E)).astype(np.float64)
    msg = rng.random((E, 3), dtype=np.float32)
    ds = TemporalGraphDataset(torch.from_numpy(src), torch.from_numpy(dst), torch.from_numpy(t),
                              torch.from_numpy(msg))
    dl = DataLoader(ds, batch_size=B, shuffle=False)
    flat = dependecyAwareBatch(dl, flat=True)
    single = get_block([0.0] * 6, [1, 1, 2, 3, 3, 5], [2, 4, 4, 1, 5, 1])
    np.savez_compressed(os.path.join(HERE, "blocks.npz"), src=src, dst=dst, t=t, batch=np.array([B]),
                        blocks=np.array(flat, dtype=np.int64), small=np.array(single, dtype=np.int64))


def capture_negs(seed):
    from neg_sampler import NegLinkSamplerDest
    rng = np.random.default_rng(seed)
    dst_nodes = np.unique(rng.integers(100, 140, size=60)).astype(np.int64)
    pos = rng.choice(dst_nodes, size=300).astype(np.int64)
    sampler = NegLinkSamplerDest(torch.from_numpy(dst_nodes))
    torch.manual_seed(1234)
    neg = sampler.sample(torch.from_numpy(pos)).numpy()
    np.savez_compressed(os.path.join(HERE, "negs.npz"), dst_nodes=dst_nodes, pos=pos, neg=neg,
                        seed=np.array([1234]))


def capture_dataset(seed):
    from temporal_dataset import TemporalGraphDataset
    from torch.utils.data import DataLoader
    rng = np.random.default_rng(seed)
    E = 37
    src = torch.from_numpy(rng.integers(0, 9, size=E).astype(np.int64))
    dst = torch.from_numpy(rng.integers(0, 9, size=E).astype(np.int64))
    t = torch.from_numpy(1.0e9 + np.sort(rng.integers(0, 5000, size=E)).astype(np.float64) + 0.37)
    msg = torch.from_numpy(rng.random((E, 4), dtype=np.float32))
    blk = list(rng.integers(0, 5, size=E))
    ds = TemporalGraphDataset(src, dst, t, msg, batch=blk)
    dl = DataLoader(ds, batch_size=10, shuffle=False)
    rec = {"src": [], "dst": [], "t": [], "msg": [], "b": [], "idx": []}
    for b in dl:
        for k in rec:
            rec[k].append(b[k].numpy())
    out = {k: np.concatenate(v) for k, v in rec.items()}
    out.update(in_src=src.numpy(), in_dst=dst.numpy(), in_t=t.numpy(), in_msg=msg.numpy(),
               in_b=np.array(blk, dtype=np.int64), t_dtype=np.array([str(rec["t"][0].dtype)]))
    np.savez_compressed(os.path.join(HERE, "dataset.npz"), **out)


def _placeholder_dgl():
    """Names model_utils.py:9-12 imports; calling any of them is an error."""
    def _no(*a, **k):
        raise RuntimeError("DGL op called during golden capture")
    dgl = types.ModuleType("dgl")
    fn = types.ModuleType("dgl.function")
    ops = types.ModuleType("dgl.ops")
    base = types.ModuleType("dgl.base")
    ops.edge_softmax = _no
    base.DGLError = RuntimeError
    dgl.function, dgl.ops, dgl.base = fn, ops, base
    dgl.NID = "_ID"
    sys.modules.update({"dgl": dgl, "dgl.function": fn, "dgl.ops": ops, "dgl.base": base})


def capture_model(seed):
    _placeholder_dgl()
    import model_utils as mu
    te = mu.TimeEncode(100)
    ts = torch.tensor([0.0, 1.0, -1.0, 3.5, 1234.0, -86_400.0, 2_678_373.0, 1.7e6,
                       -2.5e6, 9.3e8, -1.2e9 + 7.0], dtype=torch.float32).view(-1, 1)
    te_out = te(ts).detach().numpy()
    torch.manual_seed(seed)
    pred = mu.EdgePredictor(100, 100)
    B, NS = 7, 3
    hs = torch.randn(B, 100)
    hp = torch.randn(B, 100)
    hn = torch.randn(B * NS, 100)
    pos, neg = pred(hs, hp, hn, neg_samples=NS)
    torch.manual_seed(seed + 1)
    tgnn = mu.TGNN(172, 100, 50, "cpu", num_heads=8, layers=1)
    shapes = {n: np.array(p.shape) for n, p in tgnn.named_parameters()}
    ntrain = sum(p.numel() for p in tgnn.parameters() if p.requires_grad)
    out = dict(te_w=te.w.weight.detach().numpy(), te_b=te.w.bias.detach().numpy(), te_t=ts.numpy(),
               te_out=te_out, pred_hs=hs.numpy(), pred_hp=hp.numpy(), pred_hn=hn.numpy(),
               pred_pos=pos.detach().numpy(), pred_neg=neg.detach().numpy(), pred_ns=np.array([NS]),
               n_trainable=np.array([ntrain]), mem=tgnn.memory.memory.detach().numpy()[:3],
               param_names=np.array(list(shapes.keys())))
    for k, (n, p) in enumerate(pred.named_parameters()):
        out[f"pred_param_{n}"] = p.detach().numpy()
    for n, s in shapes.items():
        out[f"shape_{n}"] = s
    np.savez_compressed(os.path.join(HERE, "model.npz"), **out)


def capture_msg(seed):
    from modules.msg_func import IdentityMessage
    g = torch.Generator().manual_seed(seed)
    m = IdentityMessage(5, 3, 4)
    zs, zd, raw, te = (torch.randn(6, 3, generator=g), torch.randn(6, 3, generator=g),
                       torch.randn(6, 5, generator=g), torch.randn(6, 4, generator=g))
    out = m(zs, zd, raw, te)
    np.savez_compressed(os.path.join(HERE, "msg.npz"), zs=zs.numpy(), zd=zd.numpy(), raw=raw.numpy(),
                        te=te.numpy(), out=out.numpy(), out_channels=np.array([m.out_channels]))


def capture_link_pred(seed):
    """modules/decoder.py:12-27 LinkPredictor (sigmoid output): weights + inputs + outputs."""
    from modules.decoder import LinkPredictor
    torch.manual_seed(seed)
    lp = LinkPredictor(6)
    g = torch.Generator().manual_seed(seed + 1)
    zs, zd = torch.randn(9, 6, generator=g), torch.randn(9, 6, generator=g)
    with torch.no_grad():
        out = lp(zs, zd)
    sd = {k: v.numpy() for k, v in lp.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, "link_pred.npz"), zs=zs.numpy(), zd=zd.numpy(), out=out.numpy(),
                        **{"p_" + k.replace(".", "__"): v for k, v in sd.items()})


def _install_tgn_placeholders(ref):
    """Placeholder modules for the imports memory_module.py / msg_agg.py need beyond torch (the published
    behaviour of: PyG zeros (fill 0), PyG scatter (sum / mean / max with 0 in empty rows), torch_scatter
    scatter_max (argmax = src.size(0) in empty rows, the first index of the max otherwise, its CPU kernel),
    PyG TimeEncoder (cos(Linear(1, D)(t)))).  Returns the imported reference modules."""
    tg = types.ModuleType("torch_geometric")
    tg_nn = types.ModuleType("torch_geometric.nn")
    tg_inits = types.ModuleType("torch_geometric.nn.inits")
    tg_utils = types.ModuleType("torch_geometric.utils")

    def zeros(value):
        if value is not None:
            value.data.fill_(0)

    def scatter(src, index, dim=0, dim_size=None, reduce="sum"):
        assert dim == 0
        n = int(index.max()) + 1 if dim_size is None else dim_size
        shape = (n,) + tuple(src.shape[1:])
        idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
        if reduce in ("sum", "add"):
            return src.new_zeros(shape).scatter_add(0, idx, src)
        if reduce == "mean":
            tot = src.new_zeros(shape).scatter_add(0, idx, src)
            cnt = torch.zeros(n, dtype=src.dtype).scatter_add(0, index, torch.ones(index.shape[0], dtype=src.dtype))
            return tot / cnt.clamp(min=1).view(-1, *([1] * (src.dim() - 1)))
        if reduce == "max":
            return src.new_zeros(shape).scatter_reduce(0, idx, src, reduce="amax", include_self=False)
        raise ValueError(reduce)

    tg_inits.zeros = zeros
    tg_utils.scatter = scatter
    tg.nn, tg_nn.inits, tg.utils = tg_nn, tg_inits, tg_utils
    ts = types.ModuleType("torch_scatter")

    def scatter_max(src, index, dim=0, dim_size=None):
        assert dim == 0 and src.dim() == 1
        n = int(index.max()) + 1 if dim_size is None else dim_size
        out = src.new_zeros(n).scatter_reduce(0, index, src, reduce="amax", include_self=False)
        arg = torch.full((n,), src.shape[0], dtype=torch.long)
        hit = src == out[index]
        arg = arg.scatter_reduce(0, index[hit], torch.arange(src.shape[0])[hit], reduce="amin", include_self=True)
        return out, arg

    ts.scatter_max = scatter_max
    for name, mod in (("torch_geometric", tg), ("torch_geometric.nn", tg_nn), ("torch_geometric.nn.inits", tg_inits),
                      ("torch_geometric.utils", tg_utils), ("torch_scatter", ts)):
        sys.modules[name] = mod
    import modules  # noqa: F401  (the reference's namespace package)
    te = types.ModuleType("modules.time_enc")

    class TimeEncoder(torch.nn.Module):
        def __init__(self, out_channels):
            super().__init__()
            self.out_channels = out_channels
            self.lin = torch.nn.Linear(1, out_channels)

        def reset_parameters(self):
            self.lin.reset_parameters()

        def forward(self, t):
            return self.lin(t.view(-1, 1)).cos()

    te.TimeEncoder = TimeEncoder
    sys.modules["modules.time_enc"] = te
    from modules import memory_module, msg_agg, msg_func
    return memory_module, msg_agg, msg_func


def capture_tgn_memory(ref, aggr, updater, seed, N=40, d=5, D=8, B=12, n_train=5, n_eval=2):
    """TGNMemory (modules/memory_module.py:25-215) driven as the canonical loop drives it: per train batch
    memory(n_id) over the batch's nodes plus a few others (:116-124, _get_updated_memory), then
    update_state (:126-138, train order); then train(False) (:209-215, the flush); then eval batches
    (memory(n_id), update_state in eval order).  Timestamps strictly increase and are int64: the module
    assigns scatter-max(t) into its long last_update buffer (:150), which refuses float32 t (the cast of
    temporal_dataset.py:53) — PyG's TGN convention of integer times is what it runs with; nodes repeat
    within batches."""
    mm, ma, mf = _install_tgn_placeholders(ref)
    torch.manual_seed(seed)
    agg = ma.LastAggregator() if aggr == "last" else ma.MeanAggregator()
    mem = mm.TGNMemory(N, d, D, D, mf.IdentityMessage(d, D, D), agg, memory_updater_cell=updater)
    rng = np.random.default_rng(seed)
    out = {f"p_{k.replace('.', '__')}": v.detach().numpy().copy() for k, v in mem.state_dict().items()
           if not k.startswith("_") and k not in ("memory", "last_update")}
    nb = n_train + n_eval
    src = rng.integers(0, N, (nb, B)).astype(np.int64)
    dst = rng.integers(0, N, (nb, B)).astype(np.int64)
    src[:, 1] = src[:, 0]                              # a node twice in one batch (store ordering)
    t = (np.arange(nb * B).reshape(nb, B) * 3 + 1).astype(np.int64)
    msg = rng.random((nb, B, d), dtype=np.float32)
    extra = rng.integers(0, N, (nb, 4)).astype(np.int64)
    out.update(src=src, dst=dst, t=t, msg=msg, extra=extra, meta=np.array([N, d, D, B, n_train, n_eval]))
    mem.train()
    for b in range(nb):
        if b == n_train:
            mem.train(False)                            # the flush
            out["flush_memory"] = mem.memory.detach().numpy().copy()
            out["flush_last_update"] = mem.last_update.numpy().copy()
        s, dd = torch.from_numpy(src[b]), torch.from_numpy(dst[b])
        n_id = torch.cat([s, dd, torch.from_numpy(extra[b])]).unique()
        with torch.no_grad():
            z, lu = mem(n_id)
            out[f"b{b}_nid"] = n_id.numpy()
            out[f"b{b}_z"] = z.detach().numpy().copy()
            out[f"b{b}_lu"] = lu.detach().numpy().copy()
            mem.update_state(s, dd, torch.from_numpy(t[b]), torch.from_numpy(msg[b]))
        out[f"b{b}_memory"] = mem.memory.detach().numpy().copy()
        out[f"b{b}_last_update"] = mem.last_update.numpy().copy()
        # the stores' event times per node (src / dst direction): their layout and order
        out[f"b{b}_store_s_t"] = np.concatenate([mem.msg_s_store[j][2].numpy().astype(np.float64) for j in range(N)]
                                                or [np.zeros(0)])
        out[f"b{b}_store_s_n"] = np.array([mem.msg_s_store[j][2].numel() for j in range(N)])
        out[f"b{b}_store_d_n"] = np.array([mem.msg_d_store[j][2].numel() for j in range(N)])
    np.savez(os.path.join(HERE, f"tgn_memory_{aggr}_{updater}.npz"), **out)


def _install_transformer_conv():
    """torch_geometric.nn.TransformerConv placeholder (emb_module.py:7 imports it), restating PyG's published
    semantics for the arguments emb_module.py:21-23 passes (concat=True, beta=False, root_weight=True,
    edge_dim set): lin_key / lin_query / lin_value / lin_skip with bias, lin_edge without; messages flow
    source -> target (x_j = x[edge_index[0]], x_i = x[edge_index[1]]); key_j += lin_edge(e), value_j +=
    lin_edge(e); alpha = softmax over each target's edges of q_i·k_j / sqrt(C) (PyG softmax: exp(a - max) /
    (sum + 1e-16)), dropout on alpha in training; out_i = Σ alpha v_j, heads concatenated, + lin_skip(x_i)."""
    import math
    tg_nn = sys.modules["torch_geometric.nn"]

    class TransformerConv(torch.nn.Module):
        def __init__(self, in_channels, out_channels, heads=1, concat=True, beta=False, dropout=0.0, edge_dim=None,
                     bias=True, root_weight=True, **kwargs):
            super().__init__()
            assert concat and not beta and root_weight and edge_dim is not None
            self.heads, self.out_channels, self.dropout = heads, out_channels, dropout
            HC = heads * out_channels
            self.lin_key = torch.nn.Linear(in_channels, HC)
            self.lin_query = torch.nn.Linear(in_channels, HC)
            self.lin_value = torch.nn.Linear(in_channels, HC)
            self.lin_edge = torch.nn.Linear(edge_dim, HC, bias=False)
            self.lin_skip = torch.nn.Linear(in_channels, HC, bias=bias)

        def forward(self, x, edge_index, edge_attr):
            H, C, N = self.heads, self.out_channels, x.size(0)
            j, i = edge_index[0], edge_index[1]
            q = self.lin_query(x).view(-1, H, C)[i]
            k = self.lin_key(x).view(-1, H, C)[j]
            v = self.lin_value(x).view(-1, H, C)[j]
            e = self.lin_edge(edge_attr).view(-1, H, C)
            k = k + e
            a = (q * k).sum(-1) / math.sqrt(C)
            idx = i.view(-1, 1).expand(-1, H)
            amax = torch.full((N, H), -math.inf).scatter_reduce(0, idx, a.detach(), "amax", include_self=True)
            ex = (a - amax[i]).exp()
            den = torch.zeros(N, H).scatter_add(0, idx, ex) + 1e-16
            a = torch.nn.functional.dropout(ex / den[i], p=self.dropout, training=self.training)
            msg = (v + e) * a.unsqueeze(-1)
            out = torch.zeros(N, H, C).index_add(0, i, msg).view(N, H * C)
            return out + self.lin_skip(x)

    tg_nn.TransformerConv = TransformerConv


def capture_tgn_model(ref, seed, N=60, d=5, D=8, B=10, nb=4, lr=1e-3):
    """The reference's own model wiring (verdict r4 item 4): pyg_model_utils.py:10-36 getModel(d, D, N, 'cpu')
    called as written — TGNMemory + IdentityMessage + LastAggregator, GraphAttentionEmbedding
    (modules/emb_module.py:11-29) sharing memory.time_enc, LinkPredictor (modules/decoder.py) — and
    getOptimizer (:38-43), driven by the canonical PyG TGN batch (the sequence pyg_epoch_utils.py:106-137
    carries commented out) with the reference's LastNeighborLoader (neighbor_loader.py): n_id = unique(src, pos,
    neg) -> loader -> memory(n_id) -> gnn(z, last_update, edge_index, t[e_id], msg[e_id]) -> link_pred on
    (src, pos) and (src, neg) -> BCEWithLogits on the sigmoid outputs -> update_state -> insert -> backward ->
    Adam -> memory.detach().  Pins emb_module's rel_t = last_update[edge_index[0]] - t, edge_attr =
    [time_enc(rel_t) ‖ msg], the shared time encoder (its gradient from both uses) and the composition; the
    TransformerConv / scatter / TimeEncoder placeholders' arithmetic stays parity-unpinned.  Attention dropout is
    off (gnn.conv in eval mode; the memory trains).  Integer timestamps (TGNMemory's long last_update)."""
    _install_tgn_placeholders(ref)
    _install_transformer_conv()
    import neighbor_loader
    import pyg_model_utils
    torch.manual_seed(seed)
    model = pyg_model_utils.getModel(d, D, N, "cpu")
    opt = pyg_model_utils.getOptimizer(model, lr)
    model["gnn"].conv.train(False)
    loader = neighbor_loader.LastNeighborLoader(N, 10)
    rng = np.random.default_rng(seed)
    out = {}
    for part in ("memory", "gnn", "link_pred"):
        for k, v in model[part].state_dict().items():
            if not k.startswith("_") and k not in ("memory", "last_update"):
                out[f"p_{part}__{k.replace('.', '__')}"] = v.detach().numpy().copy()
    src = rng.integers(0, N, (nb, B)).astype(np.int64)
    dst = rng.integers(0, N, (nb, B)).astype(np.int64)
    neg = rng.integers(0, N, (nb, B)).astype(np.int64)
    src[:, 1] = src[:, 0]
    t = (np.arange(nb * B).reshape(nb, B) * 7 + 3).astype(np.int64)
    msg = rng.random((nb * B, d), dtype=np.float32)
    out.update(src=src, dst=dst, neg=neg, t=t, msg=msg, meta=np.array([N, d, D, B, nb]), lr=np.array([lr]))
    ev_t, ev_msg = torch.from_numpy(t.reshape(-1)), torch.from_numpy(msg)
    assoc = torch.empty(N, dtype=torch.long)
    crit = torch.nn.BCEWithLogitsLoss()
    named = {}
    for part in ("memory", "gnn", "link_pred"):
        for k, p in model[part].named_parameters():
            named.setdefault(p, f"{part}.{k}")
    for b in range(nb):
        for part in ("memory", "gnn", "link_pred"):
            model[part].train()
        model["gnn"].conv.train(False)
        opt.zero_grad()
        s, pd_, ng = (torch.from_numpy(x[b]) for x in (src, dst, neg))
        n_id = torch.cat([s, pd_, ng]).unique()
        n_id, edge_index, e_id, _ = loader(n_id)
        assoc[n_id] = torch.arange(n_id.size(0))
        z, last_update = model["memory"](n_id)
        z = model["gnn"](z, last_update, edge_index, ev_t[e_id], ev_msg[e_id])
        pos_out = model["link_pred"](z[assoc[s]], z[assoc[pd_]])
        neg_out = model["link_pred"](z[assoc[s]], z[assoc[ng]])
        loss = crit(pos_out, torch.ones_like(pos_out)) + crit(neg_out, torch.zeros_like(neg_out))
        model["memory"].update_state(s, pd_, torch.from_numpy(t[b]), torch.from_numpy(msg[b * B:(b + 1) * B]))
        loader.insert(s, pd_, torch.from_numpy(t[b]))
        loss.backward()
        out[f"b{b}_nid"] = n_id.numpy()
        out[f"b{b}_pos"] = pos_out.detach().view(-1).numpy()
        out[f"b{b}_neg"] = neg_out.detach().view(-1).numpy()
        out[f"b{b}_loss"] = np.array([float(loss)])
        # the shared time encoder appears under memory.time_enc and gnn.time_enc: one tensor, one gradient
        for p, name in named.items():
            if p.grad is not None:
                out[f"b{b}_g_{name.replace('.', '__')}"] = p.grad.numpy().copy()
        opt.step()
        model["memory"].detach()
        out[f"b{b}_memory"] = model["memory"].memory.detach().numpy().copy()
        out[f"b{b}_last_update"] = model["memory"].last_update.numpy().copy()
    np.savez(os.path.join(HERE, "tgn_model_wiring.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default="", help="comma-separated capture names (tgn_memory, sampler, ...)")
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, args.ref)
    torch.set_num_threads(1)
    if args.only:
        if "tgn_memory" in args.only.split(","):
            for i, (aggr, upd) in enumerate((("last", "gru"), ("mean", "gru"), ("last", "rnn"))):
                capture_tgn_memory(args.ref, aggr, upd, seed=20 + i)
        if "tgn_model" in args.only.split(","):
            capture_tgn_model(args.ref, seed=30)
        print("goldens written to", HERE)
        return
    capture_sampler(args.ref, "k4_mono", num_nodes=40, K=4, num_batches=12, batch=12, monotone=True, seed=1)
    capture_sampler(args.ref, "k4_shuffled_t", num_nodes=40, K=4, num_batches=10, batch=12, monotone=False,
                    seed=2)
    capture_sampler(args.ref, "k10_mono", num_nodes=300, K=10, num_batches=8, batch=100, monotone=True, seed=3)
    capture_blocks(4)
    capture_negs(5)
    capture_dataset(6)
    capture_model(7)
    capture_msg(8)
    capture_link_pred(9)
    for i, (aggr, upd) in enumerate((("last", "gru"), ("mean", "gru"), ("last", "rnn"))):
        capture_tgn_memory(args.ref, aggr, upd, seed=20 + i)
    capture_tgn_model(args.ref, seed=30)
    print("goldens written to", HERE)


if __name__ == "__main__":
    main()
