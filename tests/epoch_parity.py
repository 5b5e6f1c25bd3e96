"""Epoch-level runs of the TGN memory path on the oracle and on the HIP engine (test infrastructure).

The epoch follows the canonical PyG TGN loop the reference carries commented out (pyg_epoch_utils.py:106-137)
with epoch_utils.py:16-165's evaluation: per epoch memory.reset_state + neighbor_loader.reset_state
(pyg_epoch_utils.py:15-16), the train split in batches with injected negatives (dropout off), then
memory.train(False) (the flush, memory_module.py:209-215) and the val split scored TGB-style with the
batch-start state — the returned MRR is the mean over batches of the batch's mean reciprocal rank
(epoch_utils.py:113-163).  Nothing is re-synchronised between the two sides: each side runs its own
trajectory from the same initial parameters, stream and negatives.

Used by tests/test_gpu_tgn_epochs.py (HIP vs oracle) and tests/test_tgn_cpu.py (the oracle's own noise
floor: the same run with one parameter tensor moved by 1 ulp)."""
from __future__ import annotations

import numpy as np
import torch


def scaled_stream(seed: int, N: int = 1000, E: int = 3000, d: int = 172, t_max: int | None = None):
    """A wiki-shaped stream (bipartite, Zipf endpoints, d = 172) scaled to N nodes and E events; t_max None
    keeps the wiki time scale (2,678,373 s)."""
    from tgnx.synth import SHAPES, StreamShape, make_stream
    base = SHAPES["tgbl-wiki"]
    shape = StreamShape("tgbl-wiki", N, E, d, True, num_src=int(round(N * base.num_src / base.num_nodes)),
                        t_max=base.t_max if t_max is None else t_max)
    return make_stream(shape, seed=seed)


def train_negatives(stream, seed: int, epoch: int) -> np.ndarray:
    rng = np.random.default_rng([seed, epoch, 17])
    return rng.choice(stream.dst_nodes, size=stream.train_end).astype(np.int64)


def val_negatives(stream, kn: int) -> np.ndarray:
    from tgnx.synth import eval_negatives
    return eval_negatives(stream, "val", kn)


def initial_state(stream, seed: int, D: int = 100, aggr: str = "last"):
    from oracle.tgn_ref import RefTGN
    torch.manual_seed(seed)
    ref = RefTGN(stream.num_nodes, stream.shape.msg_dim, hidden=D, aggr=aggr, dropout=0.0)
    return {k: v.detach().clone() for k, v in ref.state_dict().items()}


def oracle_epochs(stream, sd: dict, seed: int, epochs: int = 2, B: int = 200, kn: int = 50, lr: float = 1e-3,
                  D: int = 100, aggr: str = "last", perturb: str | None = None) -> dict:
    """perturb: name of a parameter tensor moved by one ulp (x (1 + 2^-23)) before training (noise floor)."""
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, eval_step, mrr_per_event, train_step
    ref = RefTGN(stream.num_nodes, stream.shape.msg_dim, hidden=D, aggr=aggr, dropout=0.0)
    sd = dict(sd)
    if perturb:   # (the time encoder is shared: memory.time_enc and gnn.time_enc name the same module)
        tail = perturb.split(".time_enc.", 1)[1] if ".time_enc." in perturb else None
        for k in list(sd):
            if k == perturb or (tail is not None and k.endswith(".time_enc." + tail)):
                sd[k] = sd[k] * (1.0 + 2.0 ** -23)
    ref.load_state_dict(sd)
    opt = torch.optim.Adam(ref.parameters(), lr=lr)
    ev_t = torch.from_numpy(stream.t.astype(np.float32))
    ev_msg = torch.from_numpy(stream.msg)
    vneg = torch.from_numpy(val_negatives(stream, kn))
    out = {"loss": [], "mrr": []}
    for ep in range(epochs):
        ref.memory.reset_state()
        loader = RefLastNeighborLoader(stream.num_nodes, 10)
        neg_all = torch.from_numpy(train_negatives(stream, seed, ep))
        tot = 0.0
        for a in range(0, stream.train_end, B):
            b = min(a + B, stream.train_end)
            sl = slice(a, b)
            loss, _, _ = train_step(ref, opt, loader, ev_t, ev_msg, torch.from_numpy(stream.src[sl]),
                                    torch.from_numpy(stream.dst[sl]), neg_all[a:b], ev_t[sl], ev_msg[sl])
            tot += loss * (b - a)
        ref.memory.train(False)
        per = []
        for a in range(stream.train_end, stream.val_end, B):
            b = min(a + B, stream.val_end)
            sl = slice(a, b)
            po, no = eval_step(ref, loader, ev_t, ev_msg, torch.from_numpy(stream.src[sl]),
                               torch.from_numpy(stream.dst[sl]), vneg[a - stream.train_end:b - stream.train_end],
                               ev_t[sl], ev_msg[sl])
            per.append(float(np.mean(mrr_per_event(po, no))))
        out["loss"].append(tot)
        out["mrr"].append(float(np.mean(per)))
    return out


def hip_epochs(stream, sd: dict, seed: int, epochs: int = 2, B: int = 200, kn: int = 50, lr: float = 1e-3,
               D: int = 100, aggr: str = "last") -> dict:
    """The same epochs on the fused HIP step (TgnEngine.train_batch with injected negatives, flush, eval_batch)."""
    from tgnx.sampler import LastNeighborLoader
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    dev = torch.device("cuda")
    model = TGNModel(stream.num_nodes, stream.num_events, stream.shape.msg_dim, D, dev, ring=10, max_batch=B,
                     max_neg=kn, aggr=aggr, dropout=0.0)
    model.load_reference_state(sd)
    eng = TgnEngine(model, LastNeighborLoader(stream.num_nodes, 10, device=dev),
                    dict(src=stream.src, dst=stream.dst, t=stream.t.astype(np.float32), msg=stream.msg),
                    TgnAdam(model, lr), dst_nodes=stream.dst_nodes)
    vneg = torch.from_numpy(val_negatives(stream, kn))
    out = {"loss": [], "mrr": []}
    for ep in range(epochs):
        eng.reset_state()
        neg_all = torch.from_numpy(train_negatives(stream, seed, ep))
        l0 = eng.loss_sum()
        for a in range(0, stream.train_end, B):
            b = min(a + B, stream.train_end)
            eng.train_batch(a, b - a, neg=neg_all[a:b], dropout=False)
        eng.flush()
        per = []
        for a in range(stream.train_end, stream.val_end, B):
            b = min(a + B, stream.val_end)
            _, _, rr = eng.eval_batch(a, b - a, vneg[a - stream.train_end:b - stream.train_end])
            per.append(rr.double().mean())
        torch.cuda.synchronize()
        eng.check()
        out["loss"].append(eng.loss_sum() - l0)
        out["mrr"].append(float(torch.stack(per).mean()))
    return out
