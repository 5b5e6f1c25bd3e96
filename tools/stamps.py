"""Wave timeline of the TGN train step (diagnostic; needs a library built with -DTGNX_STAMPS, selected with
TGNX_LIB).  Replays the wiki-shaped resident step (bench.py's TGN workload) with stamping on, then reports
per launch: the active span (first wave start -> last wave end), the gap to the previous launch, wave
durations and workgroup counts.  s_memrealtime is a 100 MHz counter; each XCD's copy is aligned to XCD 0
by the median start offset of the step's first launch (tgn_mark), which has workgroups on every XCD.

  TGNX_LIB=build_var/stamps/libtgnx.so python tools/stamps.py [--steps 20] [--dataset tgbl-wiki]
"""
import argparse
import ctypes
import math
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tgb-tgn-dgl_amd"))

NAMES = {1: "tgn_mark", 2: "tgn_scan", 3: "tgn_agg_emit", 4: "tgn_attn_fwd", 5: "tgn_pred_train", 6: "tgn_attn_bwd",
         7: "tgn_adam", 20: "gemm", 21: "gemm2", 22: "gemmN", 23: "gemm_fixup"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--dataset", default="tgbl-wiki")
    ap.add_argument("--batch", type=int, default=200)
    ap.add_argument("--aggr", default="last")
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--raw", default="", help="save the raw records (.npy)")
    ap.add_argument("--bins", action="store_true", help="per block-range start / duration table")
    ap.add_argument("--top", type=int, default=0, help="per launch, the N workgroups ending last")
    args = ap.parse_args()
    args.bins_at = {}
    from tgnx import _lib
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import SHAPES, make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel

    dev = torch.device("cuda")
    shape = SHAPES[args.dataset]
    stream = make_stream(shape, seed=0)
    N, d, D, K = shape.num_nodes, shape.msg_dim, 100, 10
    model = TGNModel(N, stream.num_events, d, D, dev, ring=K, max_batch=args.batch, max_neg=1, aggr=args.aggr,
                     dropout=0.1, generator=torch.Generator().manual_seed(0), layers=args.layers)
    eng = TgnEngine(model, LastNeighborLoader(N, K, device=dev),
                    dict(src=stream.src, dst=stream.dst, t=stream.t.astype(np.float32), msg=stream.msg),
                    TgnAdam(model, 1e-4), dst_nodes=np.unique(stream.dst), seed=1234)
    eng.bind_resident(0, stream.train_end, args.batch, dropout=True)
    eng.begin_epoch()
    eng.capture_resident()
    for _ in range(args.warmup):
        eng.replay_resident()
    torch.cuda.synchronize()
    cap = 1 << 20
    buf = torch.zeros(cap * 32, dtype=torch.uint8, device=dev)
    _lib.call("tgnx_stamps_set", buf.data_ptr(), cap)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.steps):
        eng.replay_resident()
    ev1.record()
    torch.cuda.synchronize()
    n = int(_lib.lib().tgnx_stamps_count())
    _lib.call("tgnx_stamps_set", None, 0)
    step_us = ev0.elapsed_time(ev1) / args.steps * 1e3
    dt = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("kid", "<u4"), ("blk", "<u4"), ("xcc", "<u4"), ("wave", "<u4")])
    allrec = np.frombuffer(buf.cpu().numpy().tobytes(), dtype=dt).reshape(64, cap // 64)
    if n > cap // 64:
        print(f"warning: a shard overflowed ({n} > {cap // 64} records)")
    rec = allrec[:, : min(n, cap // 64)].reshape(-1)
    rec = rec[rec["t1"] > 0]
    n = rec.shape[0]
    if args.raw:
        np.save(args.raw, rec)
    print(f"{n} workgroup records over {args.steps} steps; graph replay {step_us:.1f} us/step")
    # per XCD: launches are strictly ordered on the stream, so a launch's waves on one XCD all start after
    # the previous launch's waves there have ended
    per_x = defaultdict(list)
    for r in rec:
        per_x[int(r["xcc"]) & 7].append(r)
    launches_x = {}
    for x, rs in per_x.items():
        rs.sort(key=lambda r: int(r["t0"]))
        L, cur, tmax = [], [], 0
        for r in rs:
            if cur and (int(r["t0"]) > tmax or int(r["kid"]) != int(cur[-1]["kid"]) and int(r["t0"]) >= tmax):
                L.append(cur)
                cur = []
            cur.append(r)
            tmax = max(tmax, int(r["t1"])) if len(cur) > 1 else int(r["t1"])
        if cur:
            L.append(cur)
        launches_x[x] = L
    # align XCD clocks on tgn_agg_emit launches (once per step in every step form; the pipelined step has no
    # tgn_mark launch: it marks the next batch inside tgn_pred_train)
    SK = 3
    starts = {x: [min(int(r["t0"]) for r in l) for l in L if int(l[0]["kid"]) == SK] for x, L in launches_x.items()}
    ref = starts.get(0) or next(iter(starts.values()))
    off = {}
    for x, s in starts.items():
        k = min(len(s), len(ref))
        off[x] = int(np.median(np.array(s[:k], dtype=np.int64) - np.array(ref[:k], dtype=np.int64))) if k else 0
    print("XCD clock offsets vs XCD 0 (us):", {x: round(o * 0.01, 2) for x, o in sorted(off.items())})
    # global launch list: merge per-XCD launches by aligned start
    allw = []
    for x, L in launches_x.items():
        for l in L:
            for r in l:
                allw.append((int(r["t0"]) - off[x], int(r["t1"]) - off[x], int(r["kid"]), int(r["blk"]), x,
                             int(r["wave"])))
    allw.sort()
    glaunch, cur, tmax = [], [], 0
    for w in allw:
        if cur and w[0] > tmax + 20 and (w[2] != cur[-1][2] or w[0] > tmax + 50):  # 0.2 / 0.5 us of slack
            glaunch.append(cur)
            cur = []
        cur.append(w)
        tmax = max(tmax, w[1]) if len(cur) > 1 else w[1]
    if cur:
        glaunch.append(cur)
    # fold into steps: a step starts at tgn_agg_emit (the non-pipelined step's mark / scan then close the
    # previous one)
    steps, st = [], None
    for l in glaunch:
        if l[0][2] == SK:
            st = []
            steps.append(st)
        if st is not None:
            st.append(l)
    steps = [s for s in steps if len(s) == len(steps[0])]
    if not steps:
        print("no complete steps found")
        return
    nl = len(steps[0])
    print(f"{len(steps)} steps x {nl} launches (times in us, averaged over steps)")
    print(f"{'launch':16s} {'WGs':>5s} {'busy':>5s} {'gap':>6s} {'span':>7s} {'WG p50':>7s} {'busy avg':>8s} {'WG max':>7s} "
          f"{'skew95':>7s}")
    tot_gap = tot_span = 0.0
    for i in range(nl):
        ls = [s[i] for s in steps]
        prev_end = [max(w[1] for w in s[i - 1]) if i else None for s in steps]
        gaps = [(min(w[0] for w in l) - pe) * 0.01 for l, pe in zip(ls, prev_end) if pe is not None]
        spans = [(max(w[1] for w in l) - min(w[0] for w in l)) * 0.01 for l in ls]
        wd = [(w[1] - w[0]) * 0.01 for l in ls for w in l]
        skew = [(sorted(w[0] for w in l)[int(0.95 * (len(l) - 1))] - min(w[0] for w in l)) * 0.01 for l in ls]
        wgs = np.mean([len({(w[3]) for w in l}) for l in ls])
        busy = [x for x in wd if x > 0.5]
        nbusy = len(busy) / len(ls)
        g = float(np.mean(gaps)) if gaps else 0.0
        tot_gap += g
        tot_span += float(np.mean(spans))
        print(f"{NAMES.get(ls[0][0][2], ls[0][0][2]):16s} {wgs:5.0f} {nbusy:5.0f} {g:6.2f} {np.mean(spans):7.2f} "
              f"{np.median(wd):7.2f} {np.mean(busy) if busy else 0:8.2f} {np.max(wd):7.2f} {np.mean(skew):7.2f}")
    if args.bins:
        print("per block range (blocks: WG-count, mean start offset / mean duration / max duration, us):")
        for i in range(nl):
            ls = [s[i] for s in steps]
            nb = max(w[3] for l in ls for w in l) + 1
            edges = sorted(set([0] + [int(x) for x in args.bins_at.get(i, [])] + [nb]))
            if len(edges) == 2:
                q = max(1, -(-nb // 12))
                edges = list(range(0, nb, q)) + [nb]
            parts = []
            for a, b in zip(edges[:-1], edges[1:]):
                ws = [(w[0] - min(x[0] for x in l), w[1] - w[0]) for l in ls for w in l if a <= w[3] < b]
                if ws:
                    st_, du = np.array(ws, dtype=np.float64).T * 0.01
                    parts.append(f"[{a}-{b - 1}] {st_.mean():.1f}/{du.mean():.1f}/{du.max():.1f}")
            print(f"  {i:2d} {NAMES.get(ls[0][0][2], ls[0][0][2]):14s} " + "  ".join(parts))
    if args.top:
        print(f"per launch: the {args.top} workgroups ending last (block: mean start / mean duration / mean end, us)")
        for i in range(nl):
            ls = [s[i] for s in steps]
            acc = defaultdict(list)
            for l in ls:
                t0 = min(x[0] for x in l)
                for w in l:
                    acc[w[3]].append(((w[0] - t0) * 0.01, (w[1] - w[0]) * 0.01))
            m = sorted(((b, np.mean([a for a, _ in v]), np.mean([d for _, d in v])) for b, v in acc.items()),
                       key=lambda r: -(r[1] + r[2]))[:args.top]
            print(f"  {i:2d} {NAMES.get(ls[0][0][2], ls[0][0][2]):14s} " +
                  "  ".join(f"{b}: {s_:.1f}/{d:.1f}/{s_ + d:.1f}" for b, s_, d in m))
    for i in range(nl):  # intra-kernel checkpoints (TGNX_STAMP_AT), busy workgroups
        ls = [s[i] for s in steps]
        mids = [(w[5] & 0xFFFF, w[5] >> 16, w[1] - w[0]) for l in ls for w in l if w[5]]
        if mids:
            a = np.array(mids, dtype=np.float64) * 0.01
            print(f"  checkpoints {NAMES.get(ls[0][0][2], ls[0][0][2])}: at0 {a[:, 0].mean():.2f} us, at1 "
                  f"{a[:, 1].mean():.2f} us, end {a[:, 2].mean():.2f} us (mean over {len(mids)} workgroups)")
    step_span = np.mean([(max(w[1] for w in s[-1]) - min(w[0] for w in s[0])) * 0.01 for s in steps])
    print(f"sum of spans {tot_span:.1f}, sum of gaps {tot_gap:.1f}, first start -> last end {step_span:.1f} us; "
          f"replay {step_us:.1f} us/step")


if __name__ == "__main__":
    main()
