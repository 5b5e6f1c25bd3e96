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
  link_pred.npz  modules/decoder.py:108-123  LinkPredictor (sigmoid output)
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
    """modules/decoder.py:108-123 LinkPredictor (sigmoid output): weights + inputs + outputs."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, args.ref)
    torch.set_num_threads(1)
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
    print("goldens written to", HERE)


if __name__ == "__main__":
    main()
