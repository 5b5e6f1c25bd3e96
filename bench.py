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

# the step is replayed from HIP graphs; CLR's graph packet capture (its default) left ~0.5 us more between the
# replayed launches: 0.0917 vs 0.0878 ms per step (profiles/r5/r5_graph_packet_ab.txt). Read when the HIP runtime
# initialises, so set before torch; an explicit setting wins (tgnx/__init__.py does the same for the drop-in).
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

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


def _log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _cgroup_cpus():
    """CPU quota of this process's cgroup (v2 cpu.max or v1 cfs quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def _cores() -> int:
    """Host cores this process may use (the CPU baseline uses all of them): the affinity mask,
    bounded by the cgroup's CPU quota (a GPU box's mask lists the whole machine while its quota is a share;
    threads beyond the quota only time-slice)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = _cgroup_cpus()
    return min(n, q) if q else n


def _cpu_info() -> dict:
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return {"cpu_model": _cpu_model(), "affinity_cpus": aff, "cgroup_cpu_quota": _cgroup_cpus()}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _group_size(world: int) -> int:
    """Ranks as the process group reports them (world from the environment otherwise)."""
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else world


def _metric(dataset: str, model: str) -> str:
    return (f"temporal edges/sec on {dataset} TGN (train step)" if model == "tgn" else
            f"temporal edges/sec on {dataset} TGNN, running DGL block-loop path (train step)")


def timed_window(nb_epoch, steps, warmup, mode):
    """The timed window: `steps` consecutive batches from batch `start` of the train epoch (0-based).  mid: centred
    in the epoch (rings and message stores in their steady state; an early window samples partly empty rings),
    start: right after the warmup.  Never before the warmup's end: the loop runs `prefill` untimed steps, then
    `warmup` steps, then times batches start .. start + steps - 1 (wrapping through the epoch boundaries when
    steps > nb_epoch - start; each boundary's begin_epoch is then inside the timed region)."""
    start = max(0, (nb_epoch - steps) // 2) if mode == "mid" else 0
    start = max(start, warmup)
    prefill = start - warmup
    boundaries = sum(1 for i in range(start, start + steps) if i > 0 and i % nb_epoch == 0)
    note = (f"batches {start}..{start + steps - 1} of the {nb_epoch}-batch train epoch sequence (0-based; {prefill} "
            f"untimed prefill + {warmup} warmup steps before it"
            + (f"; the window crosses {boundaries} epoch boundar{'y' if boundaries == 1 else 'ies'}, whose "
               f"begin_epoch (ring / state reset) is timed" if boundaries else "") + ")")
    return start, prefill, boundaries, note


def cpu_baseline(stream, B, budget_s=15.0, max_batches=40):
    """Oracle (faithful per-block CPU restatement, the 'port') on the same stream, bounded sample; the
    train epoch's time is extrapolated from it (stated in the sample)."""
    sys.path.insert(0, ROOT)
    from oracle import blocks_ref
    from oracle.epoch_ref import train_batch
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgnn_ref import RefTGNN
    cores = _cores()
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
        _log(f"cpu_baseline (TGNN oracle) B={B}: batch {n} {dt:.2f} s")
    timed = max(n - 1, 1)
    rate = timed * B / max(t_total, 1e-9)
    return {"value": round(rate, 2), "unit": "events/s", "cores": cores, "kind": "port", **_cpu_info(),
            "epoch_s_extrapolated": round(stream.train_end / rate, 1),
            "sample": f"oracle per-block restatement (oracle/epoch_ref.py), train batches 2..{n} of the same "
                      f"{stream.shape.name}-shaped stream, B={B}, K=10, dropout 0.6 (reference epoch 1), torch CPU "
                      f"threads={cores}; the train epoch ({stream.train_end} events) extrapolated at this rate"}


def run_tgnn(args, world, rank, dev, probe=True):
    """The running reference path (model_utils.TGNN, DGL EdgeGATConv block loop).  probe=False: the timed
    window only (the B = 2,000 config-#1 line)."""
    _log(f"tgnn: {args.dataset} B={args.batch * world}")

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
    grouped = False
    if use_graph:
        eng.capture_resident(1)
        grouped = world == 1 and hasattr(eng, "capture_group") and eng.capture_group(8)   # (as the TGN line)

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

    start, prefill, boundaries, window_note = timed_window(nb_epoch, args.steps, args.warmup, args.window)
    _log(f"tgnn: B={Bg}: timed window {window_note}")
    for _ in range(prefill + args.warmup):
        step()
    barrier()
    e0, s0 = eng.units()
    t0 = time.perf_counter()
    if grouped and boundaries == 0:   # (no epoch boundary inside the window)
        eng.replay_resident_n(args.steps)
        counter["i"] += args.steps
    else:
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

    # live kernel timing (HIP events on the launch stream) for the roofline, over the TIMED window: before each
    # kernel's probe the epoch is rewound (begin_epoch) and replayed to batch `start`, then the probe's eager steps
    # run the same batches start .. start + steps - 1 as the timed region
    bytes_edge = 20 + 4 * d + 4 * D + 4
    bytes_root = 4 * D + 4
    probes = {}
    kernels = (("tgnn_edge_fwd", 1), ("tgnn_edge_bwd", 2), ("tgnn_seg_fwd", 6), ("tgnn_seg_bwd", 8),
               ("tgnn_pred_train", 4), ("tgnn_assemble", 3), ("tgnn_meta_collapse", 9), ("tgnn_adam", 7))
    # (probes of kernels folded into another launch in this configuration record no launch and are skipped:
    # tgnn_seg_fwd below 1,000 events, in tgnn_pred_train; tgnn_adam at world 1, in tgnn_assemble)
    for name, kid in (kernels if probe and not args.no_probe else ()):
        counter["i"] = 0
        for _ in range(start):
            step()
        barrier()
        _lib.call("tgnx_probe_enable", kid)
        pe0, ps0 = eng.units()
        for _ in range(args.steps):
            step(eager=True)          # probes record events around eager launches
        barrier()
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.call("tgnx_probe_read", ctypes.byref(ms), ctypes.byref(n))
        _lib.call("tgnx_probe_enable", 0)
        pe1, ps1 = eng.units()
        if int(n.value) == 0:   # (a kernel folded into another launch in this build: nothing to time)
            continue
        launches = int(n.value)
        avg_ms = ms.value / launches
        # units per launch: edges / segments this rank's launch processed (rows are sliced per rank).
        # Edge kernels gather per edge the ring entry / edge record, feature row and neighbour memory
        # row (SURVEY §8(d) per sampled edge); segment kernels read per root its memory row + time.
        edges = (pe1 - pe0) / launches
        roots = (ps1 - ps0) / launches
        algo = edges * bytes_edge if name.startswith("tgnn_edge") else roots * bytes_root
        probes[name] = dict(avg_us=avg_ms * 1e3, launches=launches, edges=edges, roots=roots, bytes=algo,
                            gbs=algo / (avg_ms * 1e-3) / 1e9)
    blocks_mean = float(np.mean([blk[i:i + Bg].max() + 1 for i in range(0, stream.train_end, Bg)]))
    if not probes:
        return {"metric": _metric(args.dataset, "tgnn"), "value": round(args.steps * Bg / elapsed, 1),
                "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "steps": args.steps, "timed_window": window_note, "loss_sum": round(loss, 4),
                "config": {"timed_steps": [prefill + args.warmup, prefill + args.warmup + args.steps]},
                "edges_per_step": round((e1 - e0) / args.steps / world, 1),
                "segments_per_step": round((s1 - s0) / args.steps / world, 1),
                "blocks_per_batch_mean": round(blocks_mean, 1)}
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
            "metric": _metric(args.dataset, "tgnn"),
            "value": round(args.steps * Bg / elapsed, 1),
            "unit": "events/s",
            "n_gpus": _group_size(world),
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
                       "launch": ("hip-graph replay, 8 steps per graph in the timed window" if grouped and boundaries == 0
                                  else "hip-graph replay per step") if use_graph else "eager",
                       "edges_per_step": round((e1 - e0) / args.steps / world, 1),
                       "timed_batches": [start, start + args.steps - 1], "timed_window": window_note,
                       "timed_steps": [prefill + args.warmup, prefill + args.warmup + args.steps],
                       "probe_window": "the timed batches (each probe rewinds the epoch and replays to its start)",
                       "blocks_per_batch_mean": round(blocks_mean, 1)},
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



def cpu_baseline_tgn(stream, B, budget_s=45.0, aggr="last", layers=1):
    """Oracle restatement of the TGN memory path (oracle/tgn_ref.py) over ONE full train epoch of the same
    stream at batch B (BASELINE config #1: one epoch on the CPU), all affinity cores; batch 1 (empty state,
    allocator warm-up) is run but not timed.  If the epoch would exceed budget_s, the rate of the batches
    run so far is reported and the epoch time extrapolated from it (stated in the sample)."""
    sys.path.insert(0, ROOT)
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, train_step
    cores = _cores()
    torch.set_num_threads(cores)
    N, d = stream.shape.num_nodes, stream.shape.msg_dim
    torch.manual_seed(0)
    model = RefTGN(N, d, hidden=100, aggr=aggr, dropout=0.1, layers=layers)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    loader = RefLastNeighborLoader(N, 10)
    ev_t = torch.from_numpy(stream.t.astype(np.float32))
    ev_msg = torch.from_numpy(stream.msg)
    rng = np.random.default_rng(0)
    E = stream.train_end
    nb = math.ceil(E / B)
    t_total, t_first, timed_ev, n = 0.0, 0.0, 0, 0
    for n in range(nb):
        a, b = n * B, min((n + 1) * B, E)
        src, dst = torch.from_numpy(stream.src[a:b]), torch.from_numpy(stream.dst[a:b])
        neg = torch.from_numpy(rng.choice(stream.dst_nodes, size=b - a))
        t0 = time.perf_counter()
        train_step(model, opt, loader, ev_t, ev_msg, src, dst, neg, ev_t[a:b], ev_msg[a:b])
        dt = time.perf_counter() - t0
        if n == 0:
            t_first = dt
            _log(f"cpu_baseline_tgn B={B}: batch 1 {dt:.2f} s, {cores} threads")
        else:
            t_total += dt
            timed_ev += b - a
        if n % 50 == 49:
            _log(f"cpu_baseline_tgn B={B}: {n + 1}/{nb} batches, {t_total:.1f} s")
        if t_total > budget_s:
            break
    done = n + 1
    rate = timed_ev / max(t_total, 1e-9)
    full = done == nb
    out = {"value": round(rate, 2), "unit": "events/s", "cores": cores, "kind": "port", **_cpu_info(),
           "batch": B, "epoch_events": E, "batches_run": done, "full_epoch": full}
    if full:
        out["epoch_s"] = round(t_first + t_total, 2)
    else:
        out["epoch_s_extrapolated"] = round(t_first + (E - min(B, E)) / max(rate, 1e-9), 1)
    out["sample"] = (f"oracle TGN restatement (oracle/tgn_ref.py: TGNMemory + {'Mean' if aggr == 'mean' else 'Last'}"
                     f"Aggregator + GRU + TransformerConv + LinkPredictor, attention dropout 0.1), "
                     f"{'one full' if full else 'part of one'} {stream.shape.name}-shaped train epoch "
                     f"({E} events, {done}/{nb} batches of {B}); rate over batches 2..{done} (batch 1 untimed), "
                     f"torch CPU threads = {cores} (all affinity cores)"
                     + ("" if full else f"; epoch time extrapolated at this rate (budget {budget_s:.0f} s)"))
    return out


def tgn_step_bytes(d, D, K, layers):
    """SURVEY §8(d) algorithmic bytes per event of the TGN train step: forward
    B_ev = R [S (20 + 4d + 4D + 4) + 4D + 4] + 4 K 20 + (20 + 4d), R = 3 roots, S = K (1 hop) or K + K^2
    (2 hops), plus the GRU memory path 2 (56 + 8d + 12D); training counts x 2 (backward re-gathers)."""
    S = K if layers == 1 else K + K * K
    fwd = 3 * (S * (20 + 4 * d + 4 * D + 4) + 4 * D + 4) + 4 * K * 20 + (20 + 4 * d)
    gru = 2 * (56 + 8 * d + 12 * D)
    return 2 * (fwd + gru)


def tgn_launch_bytes(name, E, M, Bw, Bg, D, d, K, P, N, kvf=False):
    """Algorithmic bytes of one launch of the TGN step: E sampled edges, M sampled nodes,
    Bw this rank's events, Bg the global batch, P trainable parameters, N nodes.  kvf: the 1-hop step whose
    attention backward also sums each edge's (dk, dv) (no tgn_kv_dE launch; its dE-only GEMMs in tgn_wgrad3)."""
    Qm = 3 * D + d
    per_edge = 20 + 4 * d + 4 * D + 4                 # ring entry, msg row, neighbour row, Δt
    if name == "tgn_agg_emit":                        # edge records + Δt enc ‖ message gather + aggregate
        return M * (8 * D + 4 * d + 40 + 4 * Qm) + E * (per_edge + 4)
    if name == "tgn_gru_edge":                        # ring insert ‖ GRU ([X | memory] in, z + gates out) ‖ lin_edge
        return Bg * 4 * K * 20 + M * (4 * Qm + 4 * D + 4 * D + 16 * D) + E * (4 * d + 12 + 4 * D)
    if name == "tgn_proj":                            # z0 in, q / k / v / skip out
        return M * (4 * D + 16 * D)
    if name == "tgn_attn_bwd" and kvf:                # + per edge: (dk, dv) summed into dP, dE written
        return E * (12 * D + 8) + E * (8 * D + 4 * D)
    if name in ("tgn_attn_fwd", "tgn_attn_bwd"):      # per edge: k, v, edge rows (+ softmax terms)
        return E * (12 * D + 8)
    if name == "tgn_pred_train":                      # per event 3 embedding rows ‖ the attention of its roots
        return Bw * 12 * D + E * (12 * D + 8) + 4 * (2 * D * D + 3 * D + 1)   # (each centre's edges once)
    if name == "tgn_kv_dE":                           # (dk, dv) sums ‖ dW_edge ‖ dEnc W_e
        return E * (8 * D + 8 * D) + E * (4 * D + 4 * (D + d) + 12 + 4 * D)
    if name == "tgn_wgrad_dz0":                       # dW_proj, dW_src/dst ‖ dz0 + GRU backward
        return M * 76 * D
    if name == "tgn_wgrad3":                          # dW_gru (dG, [X | memory]) ‖ dX_enc ‖ stores (‖ dW_edge ‖ dEnc W_e)
        return (M * (16 * D + 4 * Qm + 4 * D + 16 * D) + Bg * 2 * (8 + 4 * d)
                + (E * (4 * D + 4 * (D + d) + 12 + 4 * D) if kvf else 0))
    if name == "tgn_fixup_update":                    # Adam over every parameter (p, m, v, g in; p, m, v out)
        return 28 * P
    if name == "tgn_adam":
        return 28 * P
    if name == "tgn_scan":                            # two node bitmaps, sorted node / centre lists
        return N // 4 + 8 * (M + E)
    return 0


def _pmc(workload_ok):
    """profiles/pmc_traffic.json (tools/pmc_traffic.sh on the default workload): bytes per launch."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not (workload_ok and os.path.exists(pmc)):
        return {}
    try:
        return {k: v for k, v in json.load(open(pmc)).items() if isinstance(v, dict)}
    except Exception:
        return {}


def run_tgn(args, world, rank, dev):
    """The TGN memory path (north star; SURVEY §8 a14–a16): TGNMemory + GRU, TransformerConv, LinkPredictor."""
    from tgnx import _lib
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import SHAPES, make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel

    shape = SHAPES[args.dataset]
    stream = make_stream(shape, seed=0)
    N, d, D, K = shape.num_nodes, shape.msg_dim, 100, 10
    # weak scaling: --batch events per GPU (global B x world); --global-batch: B events split over the ranks
    Bg = args.global_batch if args.global_batch else args.batch * world
    g = torch.Generator().manual_seed(0)
    model = TGNModel(N, stream.num_events, d, D, dev, ring=K, max_batch=Bg, max_neg=1,
                     aggr="mean" if args.aggr == "mean" else "last", dropout=0.0 if args.no_dropout else 0.1,
                     generator=g, layers=args.layers, updater=args.updater,
                     memory="dyrep" if args.updater == "rnn" else "tgn")
    opt = TgnAdam(model, 1e-4)
    loader = LastNeighborLoader(N, K, device=dev)
    eng = TgnEngine(model, loader, dict(src=stream.src, dst=stream.dst, t=stream.t.astype(np.float32), msg=stream.msg),
                    opt, dst_nodes=np.unique(stream.dst), seed=1234, rank=rank, world=world)
    eng.keep_grads = False    # nothing reads the gradient buffer (world 1: TGNX_TGN_NO_GRAD_STORE)
    eng.bind_resident(0, stream.train_end, Bg, dropout=not args.no_dropout)
    nb_epoch = math.ceil(stream.train_end / Bg)
    counter = {"i": 0}
    use_graph = not args.no_graph
    eng.begin_epoch()
    grouped = False
    if use_graph:
        eng.capture_resident()
        # world 1: runs of 8 steps replayed as one graph (one graph launch per 8 steps; two steps per graph measured
        # 0.0848 vs 0.0854 ms per step, profiles/r6/r6ao_tgn_pair_graph_probe.txt)
        grouped = world == 1 and hasattr(eng, "capture_group") and eng.capture_group(8)

    def step(eager=False):
        if counter["i"] % nb_epoch == 0 and counter["i"] > 0:
            eng.begin_epoch()
        if use_graph and not eager:
            eng.replay_resident()
        else:
            eng.resident_train_step()
        counter["i"] += 1

    def units():   # running sums of sampled edges / nodes (ctl[13:15]; begin_epoch does not reset them)
        eng.finish()
        torch.cuda.synchronize()
        return list(eng.units())

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    start, prefill, boundaries, window_note = timed_window(nb_epoch, args.steps, args.warmup, args.window)
    _log(f"tgn: {args.dataset} B={Bg}: timed window {window_note}")
    for _ in range(prefill + args.warmup):
        step()
    barrier()
    u0 = units()
    barrier()
    t0 = time.perf_counter()
    if grouped and boundaries == 0:   # (no epoch boundary inside the window: the steps run back to back)
        eng.replay_resident_n(args.steps)
        counter["i"] += args.steps
    else:
        for _ in range(args.steps):
            step()
    eng.finish()          # data-parallel parity-set steps: the last step's exchanged rows + Adam (else a no-op)
    barrier()
    elapsed = time.perf_counter() - t0
    u1 = units()
    # (the pipelined step prefetches: after step j the counters include batch j + 1's sampled sets, so the window
    # counts batches start + 1 .. start + K)
    win_edges, win_nodes = (u1[0] - u0[0]) / args.steps, (u1[1] - u0[1]) / args.steps
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    eng.check()
    loss = eng.loss_sum()
    assert math.isfinite(loss), "non-finite loss"
    _log(f"tgn: {args.steps} steps {elapsed * 1e3 / args.steps:.4f} ms/step; probes")
    ms_step = elapsed / args.steps * 1e3
    value = args.steps * Bg / elapsed

    # live per-launch timing: HIP events around eager launches on the launch stream, units from the device
    # counters, over the TIMED window: before each launch's probe the epoch is rewound (begin_epoch) and replayed
    # from the graphs to batch `start`, and the probe's eager steps then run the timed batches start .. start + K - 1
    # again (the pipelined step prefetches: its counters count batches start + 1 .. start + K, as the timed ones)
    Bw = Bg / world
    P = model.trainable_count()
    probes = {}
    spec = (("tgn_agg_emit", 9), ("tgn_gru_edge", 1), ("tgn_proj", 11), ("tgn_attn_fwd", 6), ("tgn_pred_train", 4),
            ("tgn_attn_bwd", 8), ("tgn_kv_dE", 10), ("tgn_wgrad_dz0", 2), ("tgn_wgrad3", 12), ("tgn_fixup_update", 5),
            ("tgn_scan", 3), ("tgn_adam", 7))

    def rewind():
        eng.begin_epoch()
        counter["i"] = 0
        for _ in range(start):
            step()
        barrier()

    for name, kid in (() if args.no_probe else spec):
        rewind()
        _lib.call("tgnx_probe_enable", kid)
        pe0, pm0 = units()
        for _ in range(args.steps):
            step(eager=True)
        eng.finish()
        barrier()
        ms, n = ctypes.c_double(), ctypes.c_int64()
        _lib.call("tgnx_probe_read", ctypes.byref(ms), ctypes.byref(n))
        _lib.call("tgnx_probe_enable", 0)
        pe1, pm1 = units()
        if int(n.value) == 0:   # no such launch in this step (1 hop: attention forward inside tgn_pred_train; scan folded)
            continue
        launches = int(n.value)
        avg_ms = ms.value / launches
        steps_n = args.steps
        E = (pe1 - pe0) / steps_n
        M = (pm1 - pm0) / steps_n
        probes[name] = dict(avg_us=avg_ms * 1e3, launches=launches, edges=E, nodes=M, steps_n=steps_n)
    if not probes:      # --no-probe (A/B timing runs): the timed window only
        return {"metric": _metric(args.dataset, "tgn"), "value": round(value, 1), "unit": "events/s",
                "n_gpus": _group_size(world), "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms_step, 4), "higher_is_better": True,
                "scaling": "strong" if args.global_batch else "weak", "vs_baseline": None, "dtype": "f32",
                "data": f"synthetic {args.dataset}-shaped stream (SURVEY.md §8d), events resident in HBM",
                "config": {"workload": f"{args.dataset} TGN memory path, batch {Bg}", "global_batch": Bg,
                           "parallelism": f"dp{world}", "layers": args.layers, "timed_window": window_note,
                           "timed_steps": [prefill + args.warmup, prefill + args.warmup + args.steps],
                           "sampled_edges_per_step": round(win_edges, 1)},
                "roofline": None, "note": "--no-probe: no per-launch probes", "loss_sum": round(loss, 4)}
    kvf = args.layers == 1 and "tgn_kv_dE" not in probes
    for name, q in probes.items():
        algo = tgn_launch_bytes(name, q["edges"], q["nodes"], Bw, Bg, D, d, K, P, N, kvf) * (
            q.pop("steps_n") / q["launches"] if name != "tgn_scan" else 1)
        q.update(bytes=algo, gbs=(algo / (q["avg_us"] * 1e-6) / 1e9) if algo else None)
    dom = max(probes, key=lambda k: probes[k]["avg_us"])        # the longest launch of the step
    pd = probes[dom]
    Qm = 3 * D + d
    flops_gru_edge = None
    if "tgn_gru_edge" in probes:
        q = probes["tgn_gru_edge"]
        flops_gru_edge = 2 * q["nodes"] * (Qm + D) * 4 * D + 2 * q["edges"] * (D + d) * D
    pmc_workload = (args.dataset == "tgbl-wiki" and args.layers == 1 and args.aggr == "last" and args.batch == 200
                    and args.updater == "gru" and not args.global_batch)
    pmc = _pmc(pmc_workload)
    step_algo = tgn_step_bytes(d, D, K, args.layers) * Bw          # per GPU per step
    # the launches of the benched step (probes that ran: the parity-set step has no separate mark / scan /
    # attention-forward / k-v / Adam launch)
    pmc_step = sum(v.get("bytes_per_launch", 0) for k, v in pmc.items() if k in probes) if pmc else None
    roofline = {
        "bound": "hbm", "kernel": dom, "achieved": round(pd["gbs"], 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(pd["gbs"] / HBM_PEAK_GBS, 5),
        "traffic": pmc.get(dom, {}).get("bytes_per_launch"),
        "avg_launch_us": round(pd["avg_us"], 3), "algo_bytes_per_launch": round(pd["bytes"]),
        "step_algo_bytes": round(step_algo),
        "step_frac": round(step_algo / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
        "pmc_step_bytes": pmc_step,
        "pmc_over_algo_step": round(pmc_step / step_algo, 3) if pmc_step else None,
        "bytes_model": "per launch: DESIGN.md §5b (bench.tgn_launch_bytes; per sampled edge 20 + 4d + 4D + 4, "
                       "SURVEY §8d, plus per-node message / GRU rows, 28 B per parameter for Adam); step: SURVEY "
                       "§8(d) B_ev(train) x events per GPU (bench.tgn_step_bytes)",
        "timing": "avg_launch_us: the kernel's own begin / end timestamps (hipExtLaunchKernelGGL start / stop "
                  "events bound to the dispatch, on its launch stream: what rocprofv3 --kernel-trace reports), "
                  "eager launches of the same step; rocprofv3 summary of the same command: profiles/r6/ (r6_kernel_stats.csv; the timed window: r6_window_kernel_stats.csv)",
        "units_window": "each probe replays the timed batches (epoch rewound and replayed to the window's start); "
                        "units are the probe's own device counters over those batches",
    }
    if flops_gru_edge:
        roofline["tgn_gru_edge_tflops"] = round(flops_gru_edge / (probes["tgn_gru_edge"]["avg_us"] * 1e-6) / 1e12, 3)
    # validation pass on the device (TGNMemory.train(False) flush, then TGB-style scoring of the first
    # val batches against the dataset's negative count): exercises the eval path at full size; MRR
    # parity against the oracle is tests/test_gpu_tgn*.py (bench may not run the oracle outside its
    # cpu_baseline leg)
    from tgnx.synth import eval_negatives
    Be = Bg // world
    nval = min(10, max(1, (stream.val_end - stream.train_end) // Be))
    negs = eval_negatives(stream, "val", shape.num_neg_eval, limit=nval * Be)
    eng.flush()
    torch.cuda.synchronize()
    tv = time.perf_counter()
    rrs = []
    for i in range(nval):
        a = stream.train_end + i * Be
        _, _, rr = eng.eval_batch(a, Be, torch.from_numpy(negs[i * Be:(i + 1) * Be]))
        rrs.append(rr.clone())
    torch.cuda.synchronize()
    tv = time.perf_counter() - tv
    eng.check()
    val = {"mrr": round(float(torch.stack(rrs).mean()), 5), "batches": nval, "negatives": int(shape.num_neg_eval),
           "events_per_s": round(nval * Be / tv, 1), "note": "synthetic stream, mid-epoch state; "
           "eval-path smoke at full size (MRR parity vs the oracle: tests/test_gpu_tgn*.py)"}
    cpu = cpu1 = cpu_tgn2000 = loop = tcsr = gpu1 = None
    _log("tgn: eval pass done")
    headline = args.dataset == "tgbl-wiki" and args.layers == 1 and args.aggr == "last" and args.updater == "gru"
    if rank == 0 and world == 1 and headline and not args.no_config1 and not args.no_probe:
        gpu1 = tgnn_config1_gpu(args, dev)
    if rank == 0 and world == 1 and headline and not args.no_train_loop:
        loop = train_loop_rate(args, dev, value)
    if rank == 0 and world == 1 and not args.no_tcsr:
        tcsr = tcsr_sampler_bench(args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_tgn(stream, Bg, aggr=args.aggr, layers=args.layers)
        if headline and Bg != 2000:
            # BASELINE #1 as written: config/TGN.yml (batch_size 2000) through pyg-mem-tgn.py, whose import block
            # (:19, :24) runs the DGL TGNN dependency-block loop (model_utils.py:61-159) — its oracle restatement
            cpu1 = cpu_baseline(stream, 2000, budget_s=25.0, max_batches=12)
            cpu1["config"] = ("BASELINE #1: tgbl-wiki, config/TGN.yml batch_size 2000, the path pyg-mem-tgn.py runs "
                              "(TGNN block loop, epoch_utils.train), CPU; sampled batches, epoch extrapolated")
            if gpu1 is not None:
                gpu1["vs_cpu_baseline_config1"] = round(gpu1["value"] / max(cpu1["value"], 1e-9), 1)
            # the TGN memory-path oracle at TGN.yml's batch (the headline model on the CPU; NOT config #1's model)
            cpu_tgn2000 = cpu_baseline_tgn(stream, 2000)
            cpu_tgn2000["config"] = ("TGN memory-path oracle (the headline model) at config/TGN.yml's batch_size "
                                     "2000, one epoch on the CPU — not BASELINE #1's model (that is the TGNN loop)")
    return {
        "metric": _metric(args.dataset, "tgn"),
        "value": round(value, 1),
        "unit": "events/s",
        "n_gpus": _group_size(world),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic {args.dataset}-shaped stream (SURVEY.md §8d), events resident in HBM",
        "config": {"workload": f"{args.dataset} TGN memory path "
                               f"({'DyRepMemory + RNNCell' if args.updater == 'rnn' else 'TGNMemory + GRUCell'}, "
                               f"IdentityMessage + "
                               f"{'Mean' if args.aggr == 'mean' else 'Last'}Aggregator, "
                               f"{'2-hop temporal attention (conv2(conv1)), ' if args.layers == 2 else ''}"
                               f"TransformerConv heads=2, "
                               f"LinkPredictor), batch {Bg} global ({Bg // world}/GPU), {K} temporal neighbours, "
                               f"D=100, d={d}, attention dropout {'off' if args.no_dropout else '0.1'}",
                   "global_batch": Bg, "parallelism": f"dp{world}",
                   "launch": ("hip-graph replay, 8 steps per graph in the timed window" if grouped and boundaries == 0
                              else "hip-graph replay per step") if use_graph else "eager",
                   "layers": args.layers,
                   "timed_batches": [start, start + args.steps - 1],
                   "timed_window": window_note,
                   "epoch_boundaries_in_window": boundaries,
                   # ordinals of the timed steps among this run's steps (0 = the first step): a kernel launched once
                   # per step has these dispatch indices in a rocprofv3 trace of the command
                   # (tools/rocprof_window.py, tools/pmc_summary.py PMC_WINDOW)
                   "timed_steps": [prefill + args.warmup, prefill + args.warmup + args.steps],
                   "sampled_edges_per_step": round(win_edges, 1),
                   "sampled_nodes_per_step": round(win_nodes, 1),
                   "probe_window_edges_per_step": round(pd["edges"], 1),
                   "probe_window_nodes_per_step": round(pd["nodes"], 1)},
        "roofline": roofline,
        "kernels_us": {k: round(v["avg_us"], 3) for k, v in probes.items()},
        "kernels_gbs": {k: round(v["gbs"], 1) for k, v in probes.items() if v["gbs"]},
        "cpu_baseline": cpu,
        "cpu_baseline_config1": cpu1,
        "gpu_tgnn_config1": gpu1,
        "cpu_baseline_tgn_b2000": cpu_tgn2000,
        "train_loop": loop,
        "tcsr_sampler": tcsr,
        "val_eval_gpu": val,
        "loss_sum": round(loss, 4),
    }


def tgnn_config1_gpu(args, dev):
    """BASELINE #1's workload on the HIP path: config/TGN.yml's batch_size 2000 (TGN.yml:27) through the TGNN
    dependency-block loop pyg-mem-tgn.py runs (epoch_utils.py:168-318, model_utils.py:61-159), one GPU, on the
    same wiki-shaped stream as cpu_baseline_config1 (~930 blocks per batch), so the two are one configuration.
    Timed window: min(K, 40) batches centred in the 56-batch epoch, graph replay; parity at this batch size:
    tests/test_gpu_tgnn_b2000.py."""
    import copy
    a = copy.copy(args)
    a.batch, a.steps, a.warmup = 2000, min(args.steps, 40), min(args.warmup, 5)
    a.dataset = "tgbl-wiki"
    r = run_tgnn(a, 1, 0, dev, probe=False)
    r.update(unit="events/s", batch=2000, dtype="f32",
             workload="tgbl-wiki TGNN (running reference path: DGL EdgeGATConv block loop), config/TGN.yml "
                      "batch_size 2000, 10 temporal neighbours, H=8, D=100, d=172, "
                      f"dropout {'off' if args.no_dropout else '0.6 (epoch-1)'}; 1x MI355X, hip-graph replay")
    _log(f"tgnn config #1 (B=2000): {r['value']:.0f} events/s, {r['ms_per_step']:.3f} ms/step")
    return r


def train_loop_rate(args, dev, engine_value, epochs=3):
    """SURVEY §8(d)'s metric as defined: train-split events per second of the `train` loop that the reference
    script calls (pyg-mem-tgn.py:57 -> pyg_epoch_utils.train, here tgnx/tgn_epoch.train after the one-line
    model-import swap), on the full synthetic tgbl-wiki-shaped stream, batch --batch, one GPU.  Each epoch
    is timed whole (reset, the graph replays, the loss read-back and the AP / AUC display); epoch 1 also
    captures the step graphs.  The reported value is the best later epoch."""
    import pyg_epoch_utils as pe
    import pyg_model_utils as pm
    from tgnx.data import getDataWithDependecyBlock
    from tgnx.neg import NegLinkSamplerDest
    from tgnx.sampler import LastNeighborLoader
    os.environ.setdefault("TGNX_EVAL_NEGS", "10")     # (no eval here; keeps the unused negative lists small)
    B = args.batch
    data, tr, va, te, ns, ev, metric = getDataWithDependecyBlock(args.dataset, {"batch_size": B})
    d, N = data.msg.shape[1], data.num_nodes
    torch.manual_seed(0)
    model = pm.getModel(d, 100, N, dev, ring=10, max_batch=B, dropout=0.0 if args.no_dropout else 0.1)
    opt = pm.getOptimizer(model, 1e-4)
    nl = LastNeighborLoader(N, 10, device=dev)
    nds = NegLinkSamplerDest(torch.unique(data.dst), device=dev)
    crit = torch.nn.BCEWithLogitsLoss()
    times, losses = [], []
    import contextlib
    import io
    for ep in range(epochs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()) as out:   # (its "ap and auc:" line; kept below)
            losses.append(pe.train(model, data.msg, tr, nl, nds, None, dev, opt, crit))
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        _log(f"train loop epoch {ep + 1}: {times[-1] * 1e3:.1f} ms, loss {losses[-1]:.2f}")
    n = tr.hi - tr.lo
    best = n / min(times[1:])
    return {"value": round(best, 1), "unit": "events/s", "events_per_epoch": n, "batch": B,
            "epoch_s": [round(t, 5) for t in times], "loss_sum": [round(x, 3) for x in losses],
            "ap_auc_line": out.getvalue().strip(), "ratio_to_engine_value": round(best / engine_value, 4),
            "note": "pyg_epoch_utils.train (tgnx/tgn_epoch.train) timed whole per epoch, best of epochs 2..; "
                    "epoch 1 includes the graph capture"}


def tcsr_sampler_bench(args, K=10, reps=20):
    """The north star's t-CSR temporal sampler (csrc/tgnx_tcsr.hip tgnx_tcsr_sample): for every event of the
    train split, its two endpoints' K most recent neighbours before the event (event-id cutoff = the
    LastNeighborLoader ring row at that event), over the whole t-CSR of the stream — TGL's per-edge sampling
    pass over an epoch.  Timed with HIP events around `reps` launches.  Algorithmic bytes per root: root id 8 +
    cutoff 8 + indptr pair 16 + the binary search's ceil(log2(deg + 1)) eids (8 B each) + the window's c <= K
    entries read (indices 8 + eid 8 + ts 4) + K outputs written (20 B each) + count 4."""
    from tgnx.synth import SHAPES, make_stream
    from tgnx.tcsr import TCSR
    out = {}
    for name, nev in (("tgbl-wiki", None), ("tgbl-comment", 8_000_000)):
        s = make_stream(SHAPES[name], seed=0, num_events=nev)
        dev = torch.device("cuda")
        g = TCSR.build(s.src, s.dst, s.t, s.num_nodes, device=dev)
        E = s.train_end
        roots = torch.from_numpy(np.concatenate([s.src[:E], s.dst[:E]])).to(dev)
        cut = torch.arange(E, dtype=torch.long, device=dev).repeat(2)
        nbr, eid, ts, cnt = g.sample_recent(roots, K, cut_eid=cut)
        torch.cuda.synchronize()
        deg = (g.indptr[roots + 1] - g.indptr[roots]).double()
        search = torch.ceil(torch.log2(deg + 1)).sum().item() * 8
        algo = roots.numel() * (8 + 8 + 16 + 4 + 20 * K) + search + 20 * float(cnt.sum())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.sample_recent(roots, K, cut_eid=cut)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        out[name] = {"roots": int(roots.numel()), "nnz": int(g.indices.numel()), "num_nodes": s.num_nodes,
                     "events": s.num_events, "us_per_launch": round(us, 2),
                     "roots_per_s": round(roots.numel() / (us * 1e-6), 1),
                     "algo_bytes_per_launch": round(algo), "gbs": round(algo / (us * 1e-6) / 1e9, 1),
                     "hbm_frac": round(algo / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        _log(f"tcsr {name}: {us:.1f} us per launch of {roots.numel()} roots, {out[name]['gbs']} GB/s")
        del g, roots, cut, nbr, eid, ts, cnt
    out["note"] = ("per launch: every train event's two endpoints (Q = 2 E_train roots), K = 10, event-id cutoff; "
                   "timed with HIP events over 20 launches (includes the allocation-free launch overhead); "
                   "tgbl-comment-shaped at N = 994,790 with 8M events (16M t-CSR entries)")
    return out


def _spawn_ranks(args) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes of this script, one per GPU (RANK =
    LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), as `torch.distributed.run --nproc-per-node N`
    would.  This parent never touches the GPU (no torch.cuda call before or after the spawn; the ranks are
    children, not an exec of this process).  Rank 0 prints the JSON line; if a rank fails, the others are
    stopped and its exit code is returned."""
    import signal
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    _log(f"spawned {args.gpus} rank processes (MASTER_PORT {port})")
    rc, stopped = 0, None
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                _log(f"rank process {procs.index(p)} exited with {code}: stopping the others")
                for q in live:
                    q.send_signal(signal.SIGTERM)
                stopped = time.monotonic()
        if stopped is not None and live and time.monotonic() - stopped > 30:
            for q in live:       # (a rank blocked inside a collective may not honour SIGTERM)
                q.kill()
            stopped = time.monotonic()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); without a torch.distributed launcher N > 1 spawns N rank processes")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=200, help="events per GPU per step (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="events per step over all GPUs (strong scaling; BASELINE #5: 'batch 600' on 8 GPUs)")
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
    ap.add_argument("--no-train-loop", action="store_true", help="skip timing the drop-in pyg_epoch_utils.train loop")
    ap.add_argument("--no-tcsr", action="store_true", help="skip the t-CSR sampler leg")
    ap.add_argument("--no-probe", action="store_true",
                    help="A/B timing runs: skip the per-launch probes (no roofline) and the secondary legs")
    ap.add_argument("--no-config1", action="store_true",
                    help="skip the GPU TGNN line at config/TGN.yml's batch_size 2000 (BASELINE #1's workload)")
    ap.add_argument("--window", choices=["mid", "start"], default="mid",
                    help="TGN timed window: K batches centred in the train epoch (mid, after untimed prefill steps) "
                         "or right after the warmup (start)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of HIP-graph replay")
    ap.add_argument("--dist-backend", default="nccl", help="rehearsal only: 'gloo' to run N>1 on one device")
    ap.add_argument("--one-device", action="store_true", help="rehearsal only: every rank on cuda:0")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        _log(f"--gpus {args.gpus} but WORLD_SIZE={world} (launcher): running {world} ranks")
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
        out["secondary_path"] = {"model": other, "workload": sec.get("config", {}).get("workload"),
                                 "value": sec["value"], "unit": sec.get("unit", "events/s"),
                                 "ms_per_step": sec["ms_per_step"], "roofline": sec.get("roofline"),
                                 "kernels_us": sec.get("kernels_us"), "cpu_baseline": sec.get("cpu_baseline")}
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
