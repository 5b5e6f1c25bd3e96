"""Benchmark: temporal edges/s of the fused TGN(N) train step on tgbl-wiki-shaped batches.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one train batch.  Headline (--model tgn, the north star): the TGN memory path
(modules/memory_module.py + msg_func/msg_agg + emb_module TransformerConv + decoder LinkPredictor,
the loop pyg_epoch_utils.py:106-137 comments out): negatives, sampler, GRU memory update of every
sampled node, attention embedding, link prediction + BCE, backward, Adam, update_state + ring
insert.  Secondary (--model tgnn): the running DGL path (epoch_utils.py:186-315, all dependency
blocks of the batch).  Synthetic wiki-shaped stream
(TGB data is not downloadable here), events resident in HBM.
Data-parallel: the global batch is B·N events, every rank replays the ring/time state of the
whole batch and computes its 1/N of the rows; gradients are all-reduced over RCCL (weak scaling).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tgb-tgn-dgl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_EDGE = None   # set from the config: SURVEY.md §8(d) per sampled edge 20 + 4d + 4D + 4
BYTES_PER_ROOT = None   # per root 4D + 4


def block_ids(src, dst, batch):
    from tgnx import _lib
    out = np.empty_like(src)
    _lib.call("tgnx_block_ids_host", src.ctypes.data, dst.ctypes.data, src.shape[0], batch, out.ctypes.data)
    return out


def cpu_baseline(stream, B, budget_s=15.0, max_batches=40):
    """Oracle (faithful per-block CPU restatement, the 'port') on the same stream, bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle import blocks_ref
    from oracle.epoch_ref import train_batch
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgnn_ref import RefTGNN
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", "16")), 16))
    torch.set_num_threads(cores)
    N, d = stream.shape.num_nodes, stream.shape.msg_dim
    torch.manual_seed(0)
    model = RefTGNN(d, 100, N)            # dropout as the reference's first epoch (0.6 / 0.6)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    loader = RefLastNeighborLoader(N, 10)
    feats = torch.from_numpy(stream.msg)
    rng = np.random.default_rng(0)
    n = 0
    t_total = 0.0
    while n < max_batches and t_total < budget_s:
        sl = slice(n * B, (n + 1) * B)
        src, dst = stream.src[sl], stream.dst[sl]
        blk = blocks_ref.block_ids(src, dst, B)
        neg = rng.choice(stream.dst_nodes, size=src.shape[0])
        args = [torch.from_numpy(x) for x in (src, dst, neg, stream.t[sl].astype(np.float32), stream.msg[sl], blk)]
        t0 = time.perf_counter()
        train_batch(model, opt, loader, feats, args[0], args[1], args[2], args[3], args[4], args[5])
        dt = time.perf_counter() - t0
        if n > 0:                         # first batch (empty ring, allocator warm-up) excluded
            t_total += dt
        n += 1
    timed = max(n - 1, 1)
    return {"value": round(timed * B / max(t_total, 1e-9), 2), "unit": "events/s", "cores": cores, "kind": "port",
            "sample": f"oracle per-block restatement (oracle/epoch_ref.py), train batches 2..{n} of the same "
                      f"wiki-shaped stream, B={B}, K=10, dropout 0.6 (reference epoch 1), torch CPU threads={cores}"}


def run_tgnn(args, world, rank, dev):
    """The running reference path (model_utils.TGNN, DGL EdgeGATConv block loop)."""

    from tgnx import _lib
    from tgnx.engine import TgnnEngine
    from tgnx.model import TGNN, getOptimizer
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import SHAPES, make_stream

    shape = SHAPES[args.dataset]
    stream = make_stream(shape, seed=0)
    N, d, D, K = shape.num_nodes, shape.msg_dim, 100, 10
    Bg = args.batch * world
    blk = block_ids(stream.src, stream.dst, Bg)
    ev = dict(src=torch.from_numpy(stream.src).to(dev), dst=torch.from_numpy(stream.dst).to(dev),
              t=torch.from_numpy(stream.t.astype(np.float32)).to(dev), blk=torch.from_numpy(blk).to(dev),
              msg=torch.from_numpy(stream.msg).to(dev))
    g = torch.Generator().manual_seed(0)
    model = TGNN(d, D, N, dev, ring=K, max_batch=Bg, max_neg=1, generator=g)
    opt = getOptimizer({"gnn": model}, 1e-4)
    loader = LastNeighborLoader(N, K, device=dev)
    dst_nodes = torch.from_numpy(np.unique(stream.dst))
    eng = TgnnEngine(model, loader, ev["msg"], opt, dst_nodes=dst_nodes, seed=1234, rank=rank, world=world)
    neg_buf = torch.zeros(stream.num_events, dtype=torch.long, device=dev)
    eng.bind_resident(ev["src"], ev["dst"], ev["t"], ev["blk"], ev["msg"], neg_buf, 0, stream.train_end, Bg,
                      dropout=not args.no_dropout)
    nb_epoch = math.ceil(stream.train_end / Bg)
    counter = {"i": 0}
    use_graph = not args.no_graph
    if use_graph:
        eng.capture_resident(1)

    def step(eager=False):
        if counter["i"] % nb_epoch == 0:
            eng.begin_epoch()
        if use_graph and not eager:
            eng.replay_resident()
        else:
            eng.resident_train_step()
        counter["i"] += 1

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    e0, s0 = eng.units()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    e1, s1 = eng.units()
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    eng.check()
    loss = eng.loss_sum()
    assert math.isfinite(loss), "non-finite loss"

    # live kernel timing (HIP events on the launch stream) for the roofline, same workload
    bytes_edge = 20 + 4 * d + 4 * D + 4
    bytes_root = 4 * D + 4
    probes = {}
    for name, kid in (("tgnn_edge_fwd", 1), ("tgnn_edge_bwd", 2), ("tgnn_seg_fwd", 6), ("tgnn_seg_bwd", 8),
                      ("tgnn_pred_train", 4), ("tgnn_assemble", 3), ("tgnn_meta_collapse", 9), ("tgnn_adam", 7)):
        _lib.call("tgnx_probe_enable", kid)
        pe0, ps0 = eng.units()
        for _ in range(args.probe_steps):
            step(eager=True)          # probes record events around eager launches
        barrier()
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.call("tgnx_probe_read", ctypes.byref(ms), ctypes.byref(n))
        _lib.call("tgnx_probe_enable", 0)
        pe1, ps1 = eng.units()
        launches = max(int(n.value), 1)
        avg_ms = ms.value / launches
        # units per launch: edges / segments this rank's launch processed (rows are sliced per rank).
        # Edge kernels gather per edge the ring entry / edge record, feature row and neighbour memory
        # row (SURVEY §8(d) per sampled edge); segment kernels read per root its memory row + time.
        edges = (pe1 - pe0) / launches
        roots = (ps1 - ps0) / launches
        algo = edges * bytes_edge if name.startswith("tgnn_edge") else roots * bytes_root
        probes[name] = dict(avg_us=avg_ms * 1e3, launches=launches, edges=edges, roots=roots, bytes=algo,
                            gbs=algo / (avg_ms * 1e-3) / 1e9)
    # roofline kernel: the slowest of the per-edge / per-segment kernels (the gather path of §8(d))
    dom = max((k for k in probes if k.startswith(("tgnn_edge", "tgnn_seg"))), key=lambda k: probes[k]["avg_us"])
    pd = probes[dom]

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(dom, {}).get("bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(stream, args.batch)

    if True:
        out = {
            "metric": "temporal edges/sec on tgbl-wiki TGN (train step)",
            "value": round(args.steps * Bg / elapsed, 1),
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic tgbl-wiki-shaped stream (SURVEY.md §8d), events resident in HBM",
            "config": {"workload": f"{args.dataset} TGNN (running reference path: DGL EdgeGATConv block loop), "
                                   f"batch {args.batch}/GPU, {K} temporal neighbours, H=8, D=100, d={d}, "
                                   f"dropout {'off' if args.no_dropout else '0.6 (epoch-1)'}",
                       "global_batch": Bg, "parallelism": f"dp{world}",
                       "launch": "hip-graph replay per step" if use_graph else "eager",
                       "edges_per_step": round((e1 - e0) / args.steps / world, 1),
                       "blocks_per_batch_mean": float(np.mean([blk[i:i + Bg].max() + 1
                                                               for i in range(0, stream.train_end, Bg)]))},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(pd["gbs"], 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(pd["gbs"] / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "avg_launch_us": round(pd["avg_us"], 3),
                         "algo_bytes_per_launch": round(pd["bytes"]),
                         "bytes_model": f"SURVEY §8(d): edge kernels {bytes_edge} B/edge (ring entry 20 + feature 4d + "
                                        f"neighbour memory 4D + time 4) x edges; segment kernels {bytes_root} B/root"},
            "kernels_us": {k: round(v["avg_us"], 3) for k, v in probes.items()},
            "cpu_baseline": cpu,
            "loss_sum": round(loss, 4),
        }
        return out



def cpu_baseline_tgn(stream, B, budget_s=15.0, max_batches=40):
    """Oracle restatement of the TGN memory path (oracle/tgn_ref.py) on the same stream, bounded sample."""
    sys.path.insert(0, ROOT)
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, train_step
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", "16")), 16))
    torch.set_num_threads(cores)
    N, d = stream.shape.num_nodes, stream.shape.msg_dim
    torch.manual_seed(0)
    model = RefTGN(N, d, hidden=100, aggr="last", dropout=0.1)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    loader = RefLastNeighborLoader(N, 10)
    ev_t = torch.from_numpy(stream.t.astype(np.float32))
    ev_msg = torch.from_numpy(stream.msg)
    rng = np.random.default_rng(0)
    n, t_total = 0, 0.0
    while n < max_batches and t_total < budget_s:
        sl = slice(n * B, (n + 1) * B)
        src, dst = torch.from_numpy(stream.src[sl]), torch.from_numpy(stream.dst[sl])
        neg = torch.from_numpy(rng.choice(stream.dst_nodes, size=src.shape[0]))
        t0 = time.perf_counter()
        train_step(model, opt, loader, ev_t, ev_msg, src, dst, neg, ev_t[sl], ev_msg[sl])
        dt = time.perf_counter() - t0
        if n > 0:
            t_total += dt
        n += 1
    timed = max(n - 1, 1)
    return {"value": round(timed * B / max(t_total, 1e-9), 2), "unit": "events/s", "cores": cores, "kind": "port",
            "sample": f"oracle TGN restatement (oracle/tgn_ref.py: TGNMemory + GRU + TransformerConv + LinkPredictor), "
                      f"train batches 2..{n} of the same wiki-shaped stream, B={B}, K=10, last aggregation, "
                      f"torch CPU threads={cores}"}


def run_tgn(args, world, rank, dev):
    """The TGN memory path (north star; SURVEY §8 a14–a16): TGNMemory + GRU, TransformerConv, LinkPredictor."""
    from tgnx import _lib
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import SHAPES, make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel

    shape = SHAPES[args.dataset]
    stream = make_stream(shape, seed=0)
    N, d, D, K = shape.num_nodes, shape.msg_dim, 100, 10
    Bg = args.batch * world
    g = torch.Generator().manual_seed(0)
    model = TGNModel(N, stream.num_events, d, D, dev, ring=K, max_batch=Bg, max_neg=1,
                     aggr="mean" if args.aggr == "mean" else "last", dropout=0.0 if args.no_dropout else 0.1,
                     generator=g, layers=args.layers, updater=args.updater,
                     memory="dyrep" if args.updater == "rnn" else "tgn")
    opt = TgnAdam(model, 1e-4)
    loader = LastNeighborLoader(N, K, device=dev)
    eng = TgnEngine(model, loader, dict(src=stream.src, dst=stream.dst, t=stream.t.astype(np.float32), msg=stream.msg),
                    opt, dst_nodes=np.unique(stream.dst), seed=1234, rank=rank, world=world)
    eng.bind_resident(0, stream.train_end, Bg, dropout=not args.no_dropout)
    nb_epoch = math.ceil(stream.train_end / Bg)
    counter = {"i": 0}
    use_graph = not args.no_graph
    eng.begin_epoch()
    if use_graph:
        eng.capture_resident()

    def step(eager=False):
        if counter["i"] % nb_epoch == 0 and counter["i"] > 0:
            eng.begin_epoch()
        if use_graph and not eager:
            eng.replay_resident()
        else:
            eng.resident_train_step()
        counter["i"] += 1

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    eng.check()
    loss = eng.loss_sum()
    assert math.isfinite(loss), "non-finite loss"

    # live per-launch timing (HIP events on the launch stream), units from the device counters
    Qm = 3 * D + d
    probes = {}
    spec = (("tgn_gru_edge", 1), ("tgn_attn_fwd", 6), ("tgn_attn_bwd", 8), ("tgn_kv_dE", 10), ("tgn_wgrad_dz0", 2),
            ("tgn_agg_emit", 9), ("tgn_scan", 3), ("tgn_pred_train", 4), ("tgn_fixup_update", 5), ("tgn_adam", 7))
    if getattr(eng, "_res_fused", False):   # world 1: Adam rides in the gradient writers (no tgn_adam launch)
        spec = tuple(x for x in spec if x[0] != "tgn_adam")
    for name, kid in spec:
        _lib.call("tgnx_probe_enable", kid)
        pe0, pm0 = eng.units()
        for _ in range(args.probe_steps):
            step(eager=True)
        barrier()
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.call("tgnx_probe_read", ctypes.byref(ms), ctypes.byref(n))
        _lib.call("tgnx_probe_enable", 0)
        pe1, pm1 = eng.units()
        if int(n.value) == 0:   # no such launch in this step (1 hop: the attention forward runs in tgn_pred_train)
            continue
        launches = int(n.value)
        avg_ms = ms.value / launches
        E = (pe1 - pe0) / launches
        M = (pm1 - pm0) / launches
        # algorithmic bytes per launch: edges carry the §8(d) per-sampled-edge record
        # (ring entry 20 + msg row 4d + neighbour memory / projections 4D + Δt 4); nodes carry their
        # message gather (2 memory rows + msg row + Δt) and GRU rows (X 4Qm, memory 4D, z 4D, gates 16D)
        per_edge = 20 + 4 * d + 4 * D + 4
        if name == "tgn_gru_edge":
            algo = M * (4 * Qm + 4 * D + 4 * D + 16 * D) + E * (4 * d + 12 + 4 * D)
        elif name == "tgn_attn_fwd":
            algo = E * (12 * D + 8)
        elif name == "tgn_attn_bwd":
            algo = E * (12 * D + 8)
        elif name == "tgn_kv_dE":
            # the (dk, dv) sums (dKV rows in, dP k/v columns out) beside dW_edge (dE + edge attrs) and
            # dEnc W_e (dE again)
            algo = E * (8 * D + 8 * D) + E * (4 * D + 4 * (D + d) + 12 + 4 * D)
        elif name == "tgn_wgrad_dz0":
            # dW_proj (dP + z0), dz0 (dP, gates, memory, dG out)
            algo = M * (16 * D + 4 * D + 16 * D + 16 * D + 8 * D + 16 * D)
        elif name == "tgn_agg_emit":
            algo = M * (8 * D + 4 * d + 40 + 4 * Qm) + E * (per_edge + 4)
        else:
            algo = 0.0
        probes[name] = dict(avg_us=avg_ms * 1e3, edges=E, nodes=M, bytes=algo,
                            gbs=(algo / (avg_ms * 1e-3) / 1e9) if algo else None)
    dom = max((k for k in probes if probes[k]["bytes"]), key=lambda k: probes[k]["avg_us"])
    pd = probes[dom]
    flops_gru_edge = None
    if "tgn_gru_edge" in probes:
        q = probes["tgn_gru_edge"]
        flops_gru_edge = 2 * q["nodes"] * (Qm + D) * 4 * D + 2 * q["edges"] * (D + d) * D
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    # the PMC passes (tools/pmc_traffic.sh) run the default workload: wiki-shaped, 1 hop, last aggregation
    pmc_workload = (args.dataset == "tgbl-wiki" and args.layers == 1 and args.aggr == "last" and args.batch == 200
                    and args.updater == "gru")
    if os.path.exists(pmc) and pmc_workload:
        try:
            traffic = json.load(open(pmc)).get(dom, {}).get("bytes_per_launch")
        except Exception:
            traffic = None
    # validation pass on the device (TGNMemory.train(False) flush, then TGB-style scoring of the first
    # val batches against the dataset's negative count): exercises the eval path at full size; MRR
    # parity against the oracle is tests/test_gpu_tgn.py (bench may not run the oracle outside its
    # cpu_baseline leg)
    from tgnx.synth import eval_negatives
    nval = min(10, max(1, (stream.val_end - stream.train_end) // args.batch))
    negs = eval_negatives(stream, "val", shape.num_neg_eval, limit=nval * args.batch)
    eng.flush()
    torch.cuda.synchronize()
    tv = time.perf_counter()
    rrs = []
    for i in range(nval):
        a = stream.train_end + i * args.batch
        _, _, rr = eng.eval_batch(a, args.batch, torch.from_numpy(negs[i * args.batch:(i + 1) * args.batch]))
        rrs.append(rr.clone())
    torch.cuda.synchronize()
    tv = time.perf_counter() - tv
    eng.check()
    val = {"mrr": round(float(torch.stack(rrs).mean()), 5), "batches": nval, "negatives": int(shape.num_neg_eval),
           "events_per_s": round(nval * args.batch / tv, 1), "note": "synthetic stream, mid-epoch state; "
           "eval-path smoke at full size (MRR parity vs the oracle: tests/test_gpu_tgn.py)"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_tgn(stream, args.batch)
    return {
        "metric": "temporal edges/sec on tgbl-wiki TGN (train step)",
        "value": round(args.steps * Bg / elapsed, 1),
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic {args.dataset}-shaped stream (SURVEY.md §8d), events resident in HBM",
        "config": {"workload": f"{args.dataset} TGN memory path "
                               f"({'DyRepMemory + RNNCell' if args.updater == 'rnn' else 'TGNMemory + GRUCell'}, "
                               f"IdentityMessage + "
                               f"{'Mean' if args.aggr == 'mean' else 'Last'}Aggregator, "
                               f"{'2-hop temporal attention (conv2(conv1)), ' if args.layers == 2 else ''}"
                               f"TransformerConv heads=2, "
                               f"LinkPredictor), batch {args.batch}/GPU, {K} temporal neighbours, D=100, d={d}, "
                               f"attention dropout {'off' if args.no_dropout else '0.1'}",
                   "global_batch": Bg, "parallelism": f"dp{world}",
                   "launch": "hip-graph replay per step" if use_graph else "eager",
                   "layers": args.layers,
                   "sampled_edges_per_step": round(probes[dom]["edges"], 1),
                   "sampled_nodes_per_step": round(probes[dom]["nodes"], 1)},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(pd["gbs"], 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(pd["gbs"] / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "avg_launch_us": round(pd["avg_us"], 3), "algo_bytes_per_launch": round(pd["bytes"]),
                     "bytes_model": "DESIGN.md §TGN: per sampled edge 20 + 4d + 4D + 4 (SURVEY §8d) plus per-node "
                                    "message / GRU rows; tgn_gru_edge also " +
                                    (f"{flops_gru_edge / (probes['tgn_gru_edge']['avg_us'] * 1e-6) / 1e12:.3f} "
                                     f"TFLOP/s fp32 MFMA" if flops_gru_edge else "")},
        "kernels_us": {k: round(v["avg_us"], 3) for k, v in probes.items()},
        "cpu_baseline": cpu,
        "val_eval_gpu": val,
        "loss_sum": round(loss, 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=200, help="events per GPU per step")
    ap.add_argument("--dataset", default="tgbl-wiki")
    ap.add_argument("--model", choices=["tgn", "tgnn"], default="tgn",
                    help="tgn: the TGN memory path (north star, headline); tgnn: the running DGL block-loop path")
    ap.add_argument("--aggr", choices=["last", "mean"], default="last")
    ap.add_argument("--layers", type=int, choices=[1, 2], default=1,
                    help="TGN attention hops (2: the comment config's 2-hop temporal attention)")
    ap.add_argument("--updater", choices=["gru", "rnn"], default="gru",
                    help="TGN memory updater (rnn: DyRepMemory memory_updater_type 'rnn')")
    ap.add_argument("--only", action="store_true", help="skip the secondary path")
    ap.add_argument("--no-dropout", action="store_true", help="train mode without dropout")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe-steps", type=int, default=100)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP-graph replay")
    ap.add_argument("--dist-backend", default="nccl", help="rehearsal only: 'gloo' to run N>1 on one device")
    ap.add_argument("--one-device", action="store_true", help="rehearsal only: every rank on cuda:0")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    run = {"tgn": run_tgn, "tgnn": run_tgnn}
    out = run[args.model](args, world, rank, dev)
    if not args.only:
        other = "tgnn" if args.model == "tgn" else "tgn"
        sec = run[other](args, world, rank, dev)
        out["secondary_path"] = {"model": other, "workload": sec["config"]["workload"], "value": sec["value"],
                                 "unit": sec["unit"], "ms_per_step": sec["ms_per_step"],
                                 "roofline": sec["roofline"], "kernels_us": sec["kernels_us"],
                                 "cpu_baseline": sec["cpu_baseline"]}
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
