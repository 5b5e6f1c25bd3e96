"""ORACLE (test infrastructure only) — the PyG TGN memory path restated (SURVEY §8 a14–a16).

Follows, in /root/reference:
  TGNMemory            modules/memory_module.py:25-215: message stores (:140-145, :180-191),
                       _compute_msg (:193-207), aggregation over [msg_s; msg_d] (:165-169),
                       GRUCell (:71-72, :172), last_update = scatter-max (:174-176), the train/eval
                       ordering of update vs store (:126-138), flush on train(False) (:209-215)
  IdentityMessage      modules/msg_func.py:12-18        pinned: tests/golden/msg.npz
  Last/MeanAggregator  modules/msg_agg.py:15-26         [ext] torch_scatter.scatter_max: ties keep the
                       first index (its CPU kernel); PyG scatter 'max'/'mean' give 0 for empty rows
  TimeEncoder          [ext] torch_geometric.nn.models.tgn.TimeEncoder: cos(Linear(1, D)(t))
                       (modules/time_enc.py is absent from the reference)
  GraphAttentionEmbedding  modules/emb_module.py:11-29 over
  TransformerConv      [ext] torch_geometric.nn.TransformerConv(in, C, heads=2, dropout=0.1, edge_dim,
                       concat=True, beta=False, root_weight=True): k_j += e, v_j += e with
                       e = lin_edge(edge_attr) (no bias), alpha = softmax_i(q_i·k_j / sqrt(C)) with
                       PyG's +1e-16 denominator, out_i = Σ alpha v_j + lin_skip(x_i)
  LinkPredictor        modules/decoder.py:12-27       pinned: tests/golden/link_pred.npz
  train / eval step    the canonical PyG TGN loop that pyg_epoch_utils.py:9-147 carries commented out
                       (:106-137): memory(n_id) -> gnn -> link_pred -> BCEWithLogits on the
                       sigmoid outputs (decoder.py:27 + pyg-mem-tgn.py criterion) -> update_state
                       -> insert -> backward -> Adam -> detach; eval per TGB's tgbl-wiki TGN example
                       (all candidates of an event scored with the batch-start state, per-event MRR).
PARITY UNPINNED for the [ext] parts: torch_geometric / torch_scatter are not installed here.
Canonical choices (documented in DESIGN.md §7): message stores keep batch order (stable sort at
memory_module.py:188), scatter_max ties resolve to the first message in [msg_s; msg_d] order.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn


class RefTimeEncoder(nn.Module):
    """[ext] PyG TimeEncoder: cos(Linear(1, D)(t)).  The argument is the exactly rounded w*t+b
    (see tgnn_ref.RefTimeEncode: the HIP kernels use fmaf)."""

    def __init__(self, out_channels: int):
        super().__init__()
        self.out_channels = out_channels
        self.lin = nn.Linear(1, out_channels)

    def forward(self, t):
        t = t.view(-1, 1)
        w = self.lin.weight.view(1, -1)
        arg = (t.double() * w.double() + self.lin.bias.double()).float()
        if torch.is_grad_enabled() and (self.lin.weight.requires_grad or t.requires_grad):
            arg = arg.detach() + (t * w + self.lin.bias - (t * w + self.lin.bias).detach())
        return torch.cos(arg)


def identity_message(z_src, z_dst, raw_msg, t_enc):
    """modules/msg_func.py:17-18."""
    return torch.cat([z_src, z_dst, raw_msg, t_enc], dim=-1)


def scatter_max_first(t, index, dim_size):
    """torch_scatter.scatter_max (CPU): max per row and the first index attaining it
    (argmax = len(t) for empty rows); PyG scatter 'max' fills empty rows with 0."""
    n = t.shape[0]
    td = t.double()            # empty stores carry int64 t (memory_module.py:141)
    mx = torch.full((dim_size,), -math.inf, dtype=torch.float64)
    if n:
        mx = mx.scatter_reduce(0, index, td, reduce="amax", include_self=True)
    arg = torch.full((dim_size,), n, dtype=torch.long)
    if n:
        hit = td == mx[index]
        arg = arg.scatter_reduce(0, index[hit], torch.arange(n)[hit], reduce="amin", include_self=True)
    mx = torch.where(arg < n, mx, torch.zeros_like(mx)).to(t.dtype)
    return mx, arg


def last_aggregate(msg, index, t, dim_size):
    """modules/msg_agg.py:15-21."""
    _, arg = scatter_max_first(t, index, dim_size)
    out = msg.new_zeros((dim_size, msg.size(-1)))
    mask = arg < msg.size(0)
    out[mask] = msg[arg[mask]]
    return out


def mean_aggregate(msg, index, t, dim_size):
    """modules/msg_agg.py:24-26 (PyG scatter mean: empty rows 0)."""
    out = msg.new_zeros((dim_size, msg.size(-1))).index_add(0, index, msg)
    cnt = torch.zeros(dim_size, dtype=msg.dtype).index_add(0, index, torch.ones(index.shape[0], dtype=msg.dtype))
    return out / cnt.clamp(min=1).unsqueeze(-1)


class RefTGNMemory(nn.Module):
    """modules/memory_module.py:25-215 with IdentityMessage and Last/Mean aggregation; the updater cell
    `memory_updater` is a GRUCell or RNNCell (memory_updater_cell, :57, :70-78).  DyRepMemory
    (:218-421) with use_src_emb_in_msg = use_dst_emb_in_msg = False computes exactly this (same update
    order :316-331 vs :126-138, messages :381-421 vs :193-207, last_update :365 vs :176, cell :259-264)."""

    def __init__(self, num_nodes, raw_msg_dim, memory_dim, time_dim, aggr="last", updater="gru",
                 use_src_emb_in_msg=False, use_dst_emb_in_msg=False):
        super().__init__()
        # DyRepMemory (memory_module.py:242-267): embeddings in the messages of update_state (:387-408)
        self.use_src_emb_in_msg, self.use_dst_emb_in_msg = bool(use_src_emb_in_msg), bool(use_dst_emb_in_msg)
        self.num_nodes, self.raw_msg_dim, self.memory_dim, self.time_dim = num_nodes, raw_msg_dim, memory_dim, time_dim
        self.out_channels = raw_msg_dim + 2 * memory_dim + time_dim
        self.time_enc = RefTimeEncoder(time_dim)
        if updater == "gru":
            self.memory_updater = nn.GRUCell(self.out_channels, memory_dim)
        elif updater == "rnn":
            self.memory_updater = nn.RNNCell(self.out_channels, memory_dim)   # tanh
        else:
            raise ValueError("Memory updater can be either 'gru' or 'rnn'.")
        self.aggr = aggr
        self.register_buffer("memory", torch.zeros(num_nodes, memory_dim))
        self.register_buffer("last_update", torch.zeros(num_nodes, dtype=torch.long))
        self.register_buffer("_assoc", torch.zeros(num_nodes, dtype=torch.long))
        self.reset_state()

    def reset_state(self):
        self.memory.zero_()
        self.last_update.zero_()
        self._reset_message_store()

    def _reset_message_store(self):                                    # :140-145
        # every node starts with an empty store (:144-145); kept sparse here, an absent key reads as
        # the empty tuple (so graphs of ~1M nodes reset in O(1))
        i = torch.empty((0,), dtype=torch.long)
        m = torch.empty((0, self.raw_msg_dim))
        self._empty = (i, i, i, m)
        self.msg_s_store = {}
        self.msg_d_store = {}

    def forward(self, n_id):                                           # :116-124
        if self.training:
            return self._get_updated_memory(n_id)
        return self.memory[n_id], self.last_update[n_id]

    def update_state(self, src, dst, t, raw_msg, embeddings=None, assoc=None):   # :126-138 (DyRep :316-329)
        n_id = torch.cat([src, dst]).unique()
        if self.training:
            self._update_memory(n_id, embeddings, assoc)
            self._update_msg_store(src, dst, t, raw_msg, self.msg_s_store)
            self._update_msg_store(dst, src, t, raw_msg, self.msg_d_store)
        else:
            self._update_msg_store(src, dst, t, raw_msg, self.msg_s_store)
            self._update_msg_store(dst, src, t, raw_msg, self.msg_d_store)
            self._update_memory(n_id, embeddings, assoc)

    def _update_memory(self, n_id, embeddings=None, assoc=None):      # :147-150 (DyRep :338-341)
        memory, last_update = self._get_updated_memory(n_id, embeddings, assoc)
        with torch.no_grad():
            self.memory[n_id] = memory.detach()
            self.last_update[n_id] = last_update.detach().long()

    def _get_updated_memory(self, n_id, embeddings=None, assoc=None):  # :152-178 (DyRep :343-367)
        self._assoc[n_id] = torch.arange(n_id.size(0))
        msg_s, t_s, src_s, _ = self._compute_msg(n_id, self.msg_s_store, embeddings, assoc)
        msg_d, t_d, src_d, _ = self._compute_msg(n_id, self.msg_d_store, embeddings, assoc)
        idx = torch.cat([src_s, src_d], dim=0)
        msg = torch.cat([msg_s, msg_d], dim=0)
        t = torch.cat([t_s, t_d], dim=0)
        agg = last_aggregate if self.aggr == "last" else mean_aggregate
        aggr = agg(msg, self._assoc[idx], t, n_id.size(0))
        memory = self.memory_updater(aggr, self.memory[n_id])
        last_update, _ = scatter_max_first(t, idx, self.num_nodes)
        return memory, last_update[n_id]

    def _update_msg_store(self, src, dst, t, raw_msg, store):         # :180-191
        n_id, perm = src.sort(stable=True)
        n_id, count = n_id.unique_consecutive(return_counts=True)
        for i, idx in zip(n_id.tolist(), perm.split(count.tolist())):
            store[i] = (src[idx], dst[idx], t[idx], raw_msg[idx])

    def _compute_msg(self, n_id, store, embeddings=None, assoc=None):  # :193-207 (DyRep :376-412)
        data = [store[i] for i in n_id.tolist() if i in store] or [self._empty]
        src, dst, t, raw = (torch.cat(x, dim=0) for x in zip(*data))
        t_rel = t - self.last_update[src]
        t_enc = self.time_enc(t_rel.to(raw.dtype))
        src_mem, dst_mem = self.memory[src], self.memory[dst]
        # DyRep (:387-408): an endpoint in n_id takes its embedding row (embeddings[assoc[node]])
        if self.use_src_emb_in_msg and embeddings is not None and src.numel():
            m = torch.isin(src, n_id)
            src_mem[m] = embeddings[assoc[src[m]]]
        if self.use_dst_emb_in_msg and embeddings is not None and dst.numel():
            m = torch.isin(dst, n_id)
            dst_mem[m] = embeddings[assoc[dst[m]]]
        msg = identity_message(src_mem, dst_mem, raw, t_enc)
        return msg, t, src, dst

    def train(self, mode: bool = True):                                # :209-215
        if self.training and not mode:
            self._update_memory(torch.arange(self.num_nodes))
            self._reset_message_store()
        return super().train(mode)


class RefTransformerConv(nn.Module):
    """[ext] torch_geometric.nn.TransformerConv, concat=True, beta=False, root_weight=True."""

    def __init__(self, in_channels, out_channels, heads, dropout, edge_dim):
        super().__init__()
        self.H, self.C, self.dropout = heads, out_channels, dropout
        self.lin_key = nn.Linear(in_channels, heads * out_channels)
        self.lin_query = nn.Linear(in_channels, heads * out_channels)
        self.lin_value = nn.Linear(in_channels, heads * out_channels)
        self.lin_edge = nn.Linear(edge_dim, heads * out_channels, bias=False)
        self.lin_skip = nn.Linear(in_channels, heads * out_channels)

    def forward(self, x, edge_index, edge_attr):
        H, C = self.H, self.C
        j, i = edge_index[0], edge_index[1]                 # flow source_to_target
        q = self.lin_query(x)[i].view(-1, H, C)
        k = self.lin_key(x)[j].view(-1, H, C)
        v = self.lin_value(x)[j].view(-1, H, C)
        e = self.lin_edge(edge_attr).view(-1, H, C)
        out, _ = transformer_attention(q, k, v, e, i, x.size(0), self.dropout if self.training else 0.0)
        return out + self.lin_skip(x)


def transformer_attention(q, k, v, e, i, N, dropout=0.0):
    """[ext] TransformerConv.message + aggregate (concat, beta False): q [E,H,C] (the destination's query per
    edge), k, v, e [E,H,C], destination index i [E].  a = q·(k+e)/sqrt(C); α = softmax per destination (max
    subtracted, + 1e-16, torch_geometric.utils.softmax); out_i = Σ α (v+e).  Returns (out [N, H*C], α [E, H])."""
    H, C = q.shape[1], q.shape[2]
    k = k + e
    a = (q * k).sum(-1) / math.sqrt(C)                  # [E, H]
    amax = torch.full((N, H), -math.inf, dtype=q.dtype).scatter_reduce(0, i.view(-1, 1).expand(-1, H), a, "amax",
                                                                         include_self=True)
    ex = (a - amax[i]).exp()
    den = torch.zeros(N, H, dtype=q.dtype).index_add(0, i, ex) + 1e-16
    alpha = ex / den[i]
    a = nn.functional.dropout(alpha, p=dropout, training=dropout > 0)
    out = (v + e) * a.unsqueeze(-1)
    out = torch.zeros(N, H, C, dtype=q.dtype).index_add(0, i, out).view(N, H * C)
    return out, alpha


class RefGraphAttentionEmbedding(nn.Module):
    """modules/emb_module.py:11-29.  layers = 2 is the build's 2-hop extension (SURVEY §8d comment
    config, "no reference parity"): conv2(conv1(x)) over the same 2-hop edge set (the sampler called
    on the 1-hop node set), sharing the edge attributes; no activation between the layers."""

    def __init__(self, in_channels, out_channels, msg_dim, time_enc, dropout=0.1, layers=1):
        super().__init__()
        self.time_enc = time_enc
        self.conv = RefTransformerConv(in_channels, out_channels // 2, 2, dropout, msg_dim + time_enc.out_channels)
        if layers == 2:
            self.conv2 = RefTransformerConv(out_channels, out_channels // 2, 2, dropout,
                                            msg_dim + time_enc.out_channels)
        self.layers = layers

    def forward(self, x, last_update, edge_index, t, msg):
        rel_t = last_update[edge_index[0]] - t
        rel_t_enc = self.time_enc(rel_t.to(x.dtype))
        edge_attr = torch.cat([rel_t_enc, msg], dim=-1)
        h = self.conv(x, edge_index, edge_attr)
        if self.layers == 2:
            h = self.conv2(h, edge_index, edge_attr)
        return h


class RefLinkPredictor(nn.Module):
    """modules/decoder.py:12-27 (returns the sigmoid)."""

    def __init__(self, in_channels):
        super().__init__()
        self.lin_src = nn.Linear(in_channels, in_channels)
        self.lin_dst = nn.Linear(in_channels, in_channels)
        self.lin_final = nn.Linear(in_channels, 1)

    def forward(self, z_src, z_dst):
        h = (self.lin_src(z_src) + self.lin_dst(z_dst)).relu()
        return self.lin_final(h).sigmoid()


class RefTGN(nn.Module):
    """pyg_model_utils.py:10-36: memory + gnn (sharing memory.time_enc) + link_pred."""

    def __init__(self, num_nodes, msg_dim, hidden=100, aggr="last", dropout=0.1, layers=1, updater="gru",
                 use_src_emb_in_msg=False, use_dst_emb_in_msg=False):
        super().__init__()
        self.memory = RefTGNMemory(num_nodes, msg_dim, hidden, hidden, aggr, updater, use_src_emb_in_msg,
                                   use_dst_emb_in_msg)
        self.gnn = RefGraphAttentionEmbedding(hidden, hidden, msg_dim, self.memory.time_enc, dropout, layers)
        self.link_pred = RefLinkPredictor(hidden)
        self.layers = layers


def sample_hops(model: RefTGN, loader, n_id):
    """1 hop: loader(n_id); 2 hops (layers = 2): loader(loader(n_id).nodes) — the edges into every
    1-hop node, whose node set contains the 1-hop set."""
    n_id, ei, e_id, _ = loader(np.asarray(n_id))
    if model.layers == 2:
        n_id, ei, e_id, _ = loader(n_id)
    return torch.from_numpy(n_id), torch.from_numpy(ei), torch.from_numpy(e_id)


def _emb_args(model: RefTGN, z, assoc):
    """DyRepMemory.update_state's (embeddings, assoc) (memory_module.py:316-317): the batch's embeddings over
    its sampled node set and the loop's node -> row map, when the memory uses them in messages.  Which
    embeddings a DyRep loop passes is that loop's choice (the reference contains none; TGB's DyRep example
    [ext] passes the batch's GNN output): here the same forward's, detached (the update does not reach the
    batch's loss)."""
    mem = model.memory
    if mem.use_src_emb_in_msg or mem.use_dst_emb_in_msg:
        return z.detach(), assoc
    return ()


def train_step(model: RefTGN, opt, loader, ev_t, ev_msg, src, pos, neg, t, msg):
    """One canonical TGN train batch.  loader: oracle.sampler_ref.RefLastNeighborLoader;
    ev_t / ev_msg: the stream's t / msg (rows = e_id).  Returns (loss, pos_out, neg_out)."""
    model.train()
    opt.zero_grad()
    n_id, ei, e_id = sample_hops(model, loader, torch.cat([src, pos, neg]).unique().numpy())
    assoc = torch.zeros(model.memory.num_nodes, dtype=torch.long)
    assoc[n_id] = torch.arange(n_id.size(0))
    z, last_update = model.memory(n_id)
    z = model.gnn(z, last_update, ei, ev_t[e_id], ev_msg[e_id])
    pos_out = model.link_pred(z[assoc[src]], z[assoc[pos]])
    neg_out = model.link_pred(z[assoc[src]], z[assoc[neg]])
    crit = nn.BCEWithLogitsLoss()
    loss = crit(pos_out, torch.ones_like(pos_out)) + crit(neg_out, torch.zeros_like(neg_out))
    model.memory.update_state(src, pos, t, msg, *_emb_args(model, z, assoc))
    loader.insert(src.numpy(), pos.numpy(), t.numpy())
    loss.backward()
    opt.step()
    return float(loss.detach()), pos_out.detach().view(-1), neg_out.detach().view(-1)


def train_step_dp(model: RefTGN, opt, loader, ev_t, ev_msg, src, pos, neg, t, msg, rank: int, world: int):
    """train_step decomposed over `world` ranks the way the HIP step shards it: rank r
    takes the events [B r / W, B (r + 1) / W) as roots (memory(n_id), embedding, prediction, its share
    of the global-batch mean loss); gradients are summed with an all-reduce; the message stores and the
    ring insert replay the whole global batch on every rank; the GRU rows of the slice's src ∪ dst are
    exchanged with an all-gather of (node, last_update, memory) and written by every rank.  Returns
    (global loss, pos_out, neg_out of the slice)."""
    import torch.distributed as dist
    B = src.numel()
    lo, hi = B * rank // world, B * (rank + 1) // world
    s_src, s_pos, s_neg = src[lo:hi], pos[lo:hi], neg[lo:hi]
    model.train()
    opt.zero_grad()
    n_id, ei, e_id = sample_hops(model, loader, torch.cat([s_src, s_pos, s_neg]).unique().numpy())
    assoc = torch.zeros(model.memory.num_nodes, dtype=torch.long)
    assoc[n_id] = torch.arange(n_id.size(0))
    z, last_update = model.memory(n_id)
    z = model.gnn(z, last_update, ei, ev_t[e_id], ev_msg[e_id])
    pos_out = model.link_pred(z[assoc[s_src]], z[assoc[s_pos]])
    neg_out = model.link_pred(z[assoc[s_src]], z[assoc[s_neg]])
    bce = nn.functional.binary_cross_entropy_with_logits
    loss = (bce(pos_out, torch.ones_like(pos_out), reduction="sum")
            + bce(neg_out, torch.zeros_like(neg_out), reduction="sum")) / B
    mem = model.memory
    u = torch.cat([s_src, s_pos]).unique()
    with torch.no_grad():
        m_u, lu_u = mem._get_updated_memory(u)                          # before this batch's stores
    mem._update_msg_store(src, pos, t, msg, mem.msg_s_store)
    mem._update_msg_store(pos, src, t, msg, mem.msg_d_store)
    loader.insert(src.numpy(), pos.numpy(), t.numpy())
    loss.backward()
    lt = loss.detach().clone()
    if world > 1:
        for p in model.parameters():
            if p.grad is not None:
                dist.all_reduce(p.grad)
        dist.all_reduce(lt)
    opt.step()
    cap = 2 * (-(-B // world))
    node = torch.full((cap,), -1, dtype=torch.long)
    node[:u.numel()] = u
    lu = torch.zeros(cap, dtype=torch.long)
    lu[:u.numel()] = lu_u.long()
    rows = torch.zeros(cap, mem.memory_dim)
    rows[:u.numel()] = m_u.detach()
    if world > 1:
        g_node = [torch.empty_like(node) for _ in range(world)]
        g_lu = [torch.empty_like(lu) for _ in range(world)]
        g_rows = [torch.empty_like(rows) for _ in range(world)]
        dist.all_gather(g_node, node)
        dist.all_gather(g_lu, lu)
        dist.all_gather(g_rows, rows)
        node, lu, rows = torch.cat(g_node), torch.cat(g_lu), torch.cat(g_rows)
    ok = node >= 0
    with torch.no_grad():
        mem.memory[node[ok]] = rows[ok]
        mem.last_update[node[ok]] = lu[ok]
    return float(lt), pos_out.detach().view(-1), neg_out.detach().view(-1)


@torch.no_grad()
def eval_step(model: RefTGN, loader, ev_t, ev_msg, src, pos, negs, t, msg):
    """TGB-style eval of one batch: every event's [pos, negs...] scored against the batch-start
    memory / ring state, then update_state + insert.  Returns (pos_out [B], neg_out [B, K'])."""
    model.eval()
    cand = torch.cat([pos.view(-1, 1), negs], dim=1)            # [B, 1 + K']
    n_id, ei, e_id = sample_hops(model, loader, torch.cat([src, cand.reshape(-1)]).unique().numpy())
    assoc = torch.zeros(model.memory.num_nodes, dtype=torch.long)
    assoc[n_id] = torch.arange(n_id.size(0))
    z, last_update = model.memory(n_id)
    z = model.gnn(z, last_update, ei, ev_t[e_id], ev_msg[e_id])
    zs = z[assoc[src]].unsqueeze(1).expand(-1, cand.shape[1], -1)
    y = model.link_pred(zs.reshape(-1, z.shape[1]), z[assoc[cand.reshape(-1)]]).view(cand.shape)
    model.memory.update_state(src, pos, t, msg, *_emb_args(model, z, assoc))
    loader.insert(src.numpy(), pos.numpy(), t.numpy())
    return y[:, 0].clone(), y[:, 1:].clone()


def mrr_per_event(pos_out, neg_out):
    """TGB rank rule per event (pessimistic/optimistic average), mean reciprocal rank."""
    p = pos_out.view(-1, 1)
    opt = (neg_out > p).sum(1).double()
    pes = (neg_out >= p).sum(1).double()
    rank = 0.5 * (opt + pes) + 1
    return (1.0 / rank).numpy()
