"""ORACLE (test infrastructure only) — torch-CPU restatement of the running reference model.

Follows /root/reference/model_utils.py:
  TGNN.__init__ / forward   :14-49, :61-159   per-dependency-block loop
  EdgePredictor             :165-195          (tile pairing quirk of :192 kept)
  TimeEncode                :201-237          w = 10^-linspace(0,9,D), b = 0
  MemoryModule              :240-271          memory = ones, never written on this path
  TemporalEdgePreprocess    :422-455
  EdgeGATConv               :471-612          (ft has shape [N,H,1]: msg_fn :560-563)
  TemporalTransformerConv   :615-697          feat_drop = attn_drop = 0.6, residual, head mean
and dgl_utils.py:3-8 (`getGraph` appends one self-loop per node after the sampled edges).

The DGL operations are restated from DGL's documented semantics (DGL is not
installed here, so this part is PARITY UNPINNED against DGL itself):
  in_subgraph(g, nodes)  -> all nodes kept, the in-edges of `nodes` (edge-id order)
  edge_softmax           -> softmax over each destination's in-edges, per head
  update_all(copy, sum)  -> per-destination sum, zero for nodes with no in-edge
  add_edges              -> appended after existing edge ids

Parameter names match the reference's state_dict (tests/golden/model.npz).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class RefGraph:
    """Minimal COO graph standing in for the DGL graph built at epoch_utils.py:254."""

    def __init__(self, src, dst, nid, self_loop=True):
        M = int(nid.shape[0])
        src = src.long()
        dst = dst.long()
        if self_loop:
            loop = torch.arange(M, dtype=torch.long)
            src = torch.cat([src, loop])
            dst = torch.cat([dst, loop])
        self.src, self.dst, self.nid, self.num_nodes = src, dst, nid, M

    def add_edges(self, u, v):
        self.src = torch.cat([self.src, u.long()])
        self.dst = torch.cat([self.dst, v.long()])

    def in_edges_of(self, nodes):
        mark = torch.zeros(self.num_nodes, dtype=torch.bool)
        mark[nodes] = True
        return mark[self.dst].nonzero(as_tuple=True)[0]


class RefTimeEncode(nn.Module):
    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension
        self.w = nn.Linear(1, dimension)
        self.w.weight = nn.Parameter(torch.from_numpy(1 / 10 ** np.linspace(0, 9, dimension))
                                     .float().reshape(dimension, -1))
        self.w.bias = nn.Parameter(torch.zeros(dimension).float())

    def forward(self, t):
        # cos(Linear(1,D)(t)).  torch-CPU's addmm rounds w*t+b with an FMA on its vectorised rows but
        # not on tail rows (probe in DESIGN.md §Oracle), so the reference's argument is only defined
        # to +-1 ulp; at dt ~ 1e6 that is up to 0.25 rad on the highest-frequency dims.  The oracle
        # fixes the argument to the exactly-rounded FMA (double product is exact for fp32 inputs),
        # i.e. torch's vectorised path — the rounding the HIP kernel's fmaf reproduces.
        w = self.w.weight.view(1, -1)
        arg = (t.double() * w.double() + self.w.bias.double()).float()
        if torch.is_grad_enabled() and (self.w.weight.requires_grad or t.requires_grad):
            # same value, autograd through the fp32 graph
            arg = arg.detach() + (t * w + self.w.bias - (t * w + self.w.bias).detach())
        return torch.cos(arg)


class RefEdgePredictor(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.src_fc = nn.Linear(dim_in, dim_out)
        self.dst_fc = nn.Linear(dim_in, dim_out)
        self.out_fc = nn.Linear(dim_out, 1)

    def forward(self, h_src, h_pos_dst, h_neg_dst, neg_samples=1):
        h_src = self.src_fc(h_src)
        h_pos = F.relu(h_src + self.dst_fc(h_pos_dst))
        h_neg = F.relu(h_src.tile(neg_samples, 1) + self.dst_fc(h_neg_dst))
        return self.out_fc(h_pos), self.out_fc(h_neg)


class _Memory(nn.Module):
    def __init__(self, n, d):
        super().__init__()
        self.last_update_t = nn.Parameter(torch.zeros(n), requires_grad=False)
        self.memory = nn.Parameter(torch.ones(n, d), requires_grad=False)


class _EdgeGAT(nn.Module):
    def __init__(self, node_feats, edge_feats, out_feats, heads):
        super().__init__()
        self.fc_node = nn.Linear(node_feats, out_feats * heads)
        self.fc_edge = nn.Linear(edge_feats, out_feats * heads)
        self.attn_l = nn.Parameter(torch.empty(1, heads, out_feats))
        self.attn_r = nn.Parameter(torch.empty(1, heads, out_feats))
        self.attn_e = nn.Parameter(torch.empty(1, heads, out_feats))
        gain = nn.init.calculate_gain("relu")
        for p in (self.fc_node.weight, self.fc_edge.weight, self.attn_l, self.attn_r, self.attn_e):
            nn.init.xavier_normal_(p, gain=gain)


class _Conv(nn.Module):
    def __init__(self, ef_dim, D, H):
        super().__init__()
        self.edge_gatconv = _EdgeGAT(D, ef_dim + D, D, H)


class RefTGNN(nn.Module):
    """`TGNN` with the block loop of model_utils.py:61-159.

    feat_drop / attn_drop default to the reference's hard-coded 0.6 (:664-665); parity
    tests pass 0.0 because dropout RNG streams cannot be shared with the HIP path.
    """

    def __init__(self, ef_dim, hidden_dim, num_nodes, num_heads=8, feat_drop=0.6, attn_drop=0.6):
        super().__init__()
        D, H = hidden_dim, num_heads
        self.D, self.H, self.ef_dim = D, H, ef_dim
        self.time_assoc = torch.zeros(num_nodes)
        self.memory = _Memory(num_nodes, D)
        self.temporal_encoder = RefTimeEncode(D)
        self.embedding_attn = _Conv(ef_dim, D, H)
        self.predictor = RefEdgePredictor(D, D)
        self.feat_drop = nn.Dropout(feat_drop)
        self.attn_drop = nn.Dropout(attn_drop)

    # EdgeGATConv.forward (:565-612) + TemporalTransformerConv.forward (:688-697) on the
    # in-subgraph given as (edge ids of g, g) -> embeddings of all g nodes [M, D]
    def _embed(self, g, sub_e, ef, bt, node_ts, nfeat):
        gat = self.embedding_attn.edge_gatconv
        src, dst = g.src[sub_e], g.dst[sub_e]
        M, H, D = g.num_nodes, self.H, self.D
        tdiff = bt[sub_e] - node_ts[src]                                # :442
        efeat = torch.cat([ef[sub_e], self.temporal_encoder(tdiff)], dim=1)   # :447-448
        nfeat = self.feat_drop(nfeat)                                   # :579
        efeat = self.feat_drop(efeat)                                   # :580
        node_feat = gat.fc_node(nfeat).view(-1, H, D)
        edge_feat = gat.fc_edge(efeat).view(-1, H, D)
        el = (node_feat * gat.attn_l).sum(-1, keepdim=True)
        er = (node_feat * gat.attn_r).sum(-1, keepdim=True)
        ee = (edge_feat * gat.attn_e).sum(-1, keepdim=True)
        el_prime = el[src] + ee                                         # u_add_e :594
        e = F.leaky_relu(el_prime + er[dst], 0.2)                       # e_add_v :595-596
        # edge_softmax per destination and head (:597)
        emax = torch.full((M, H, 1), -float("inf")).scatter_reduce(0, dst.view(-1, 1, 1).expand_as(e), e,
                                                                      "amax", include_self=True)
        ex = torch.exp(e - emax[dst])
        den = torch.zeros(M, H, 1).index_add(0, dst, ex)
        a = self.attn_drop(ex / den[dst])
        ft = torch.zeros(M, H, 1).index_add(0, dst, a * el_prime)       # update_all sum :599
        rst = ft + nfeat.view(M, -1, D)                                 # Identity residual :601-604
        return rst.mean(1)                                              # :693

    def forward(self, g, ef, bt, blocks, neg_samples=1):
        bt = bt.view(-1, 1)
        s, p, n, t, m, assoc = blocks
        s_emb, p_emb, n_emb = [], [], []
        for idx, tidx in enumerate(t):
            if n[idx].dim() > 1:                                        # eval (:77-79)
                self.time_assoc[:] = tidx.max()
            else:
                self.time_assoc[n[idx]] = tidx
            self.time_assoc[p[idx]] = tidx
            self.time_assoc[s[idx]] = tidx
            pos_roots = torch.cat([s[idx], p[idx]]).unique()
            roots = torch.cat([pos_roots, n[idx].view(-1)]).unique()
            sub_e = g.in_edges_of(assoc[roots])
            node_ts = self.time_assoc[g.nid].view(-1, 1)
            nfeat = self.memory.memory[g.nid]
            embed = self._embed(g, sub_e, ef, bt, node_ts, nfeat)
            s_emb.append(embed[assoc[s[idx]]])
            p_emb.append(embed[assoc[p[idx]]])
            n_emb.append(embed[assoc[n[idx].reshape(-1)]])
            g.add_edges(assoc[s[idx]], assoc[p[idx]])                   # :151-152
            g.add_edges(assoc[p[idx]], assoc[s[idx]])
            ef = torch.cat([ef, m[idx], m[idx]], dim=0)                 # :156-157
            bt = torch.cat([bt, tidx.view(-1, 1), tidx.view(-1, 1)], dim=0)
        return self.predictor(torch.cat(s_emb), torch.cat(p_emb), torch.cat(n_emb), neg_samples=neg_samples)


def collapsed_params(model: RefTGNN) -> dict:
    """Per-head projections the HIP path runs on (exact up to fp reassociation):
    U_l = attn_l·W_n, U_r = attn_r·W_n, U_e = attn_e·W_e and the matching bias dots."""
    gat = model.embedding_attn.edge_gatconv
    H, D = model.H, model.D
    Wn = gat.fc_node.weight.view(H, D, -1)
    We = gat.fc_edge.weight.view(H, D, -1)
    return {
        "U_l": torch.einsum("hd,hdk->hk", gat.attn_l[0], Wn),
        "U_r": torch.einsum("hd,hdk->hk", gat.attn_r[0], Wn),
        "U_e": torch.einsum("hd,hdk->hk", gat.attn_e[0], We),
        "c_l": (gat.attn_l[0] * gat.fc_node.bias.view(H, D)).sum(-1),
        "c_r": (gat.attn_r[0] * gat.fc_node.bias.view(H, D)).sum(-1),
        "c_e": (gat.attn_e[0] * gat.fc_edge.bias.view(H, D)).sum(-1),
    }
