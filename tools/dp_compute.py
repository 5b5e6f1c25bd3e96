"""Per-rank compute of the data-parallel TGN step on ONE device (no collective): rank 0 of a W-rank step
(global batch W x B, this rank's B-event slice; the ring insert / store update / plans replay the global
batch) with the exchange replaced by a no-op, graph replay as bench.py.  The time per step is the DP step's
compute floor at W (the all-reduce of [gradients | row slots] comes on top); numerics are not those of a
real W-rank run (the exchange is skipped).  Prints one JSON line.
    python tools/dp_compute.py [--worlds 1 2 4 8] [--batch 200] [--steps 200] [--dataset tgbl-wiki]"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tgb-tgn-dgl_amd")]

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")  # as bench.py (before the first HIP call)

import numpy as np  # noqa: E402
import torch  # noqa: E402


_STREAMS = {}


def run(W, B, steps, warmup, dataset, layers, global_batch=0):
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import SHAPES, make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    shape = SHAPES[dataset]
    if dataset not in _STREAMS:   # (the full tgbl-comment stream takes a while to draw: once per dataset)
        print(f"[dp_compute] drawing the {dataset} stream", file=sys.stderr, flush=True)
        _STREAMS[dataset] = make_stream(shape, seed=0)
    print(f"[dp_compute] {dataset} W={W}", file=sys.stderr, flush=True)
    s = _STREAMS[dataset]
    dev = torch.device("cuda")
    Bg = global_batch if global_batch else B * W
    model = TGNModel(shape.num_nodes, s.num_events, shape.msg_dim, 100, dev, ring=10, max_batch=Bg, max_neg=1,
                     dropout=0.1, layers=layers, generator=torch.Generator().manual_seed(0))
    eng = TgnEngine(model, LastNeighborLoader(shape.num_nodes, 10, device=dev),
                    dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg), TgnAdam(model, 1e-4),
                    dst_nodes=np.unique(s.dst), seed=1234, rank=0, world=W)
    if W > 1:
        eng.exchange = lambda comm, async_op: None
    eng.bind_resident(0, s.train_end, Bg, dropout=True)
    eng.begin_epoch()
    eng.capture_resident()
    nb = math.ceil(s.train_end / Bg)
    i = 0

    def step():
        nonlocal i
        if i % nb == 0 and i > 0:
            eng.begin_epoch()
        eng.replay_resident()
        i += 1
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    eng.check()
    out = {"world": W, "global_batch": Bg, "events_per_rank": -(-Bg // W), "ms_per_step": round(ms, 4),
           "comm_floats": 0 if eng.comm is None else int(eng.comm.numel())}
    if eng.comm is not None:   # the exchange payload: gradients (+ loss slot) and W row slots of xcap rows
        G = model.grad_flat.numel()
        rows = eng.comm.numel() - G
        out.update(grad_floats=G, row_slot_floats=rows, row_slots_per_rank=eng.xcap, row_floats=model.D + 4,
                   fused_allreduce_bytes=4 * eng.comm.numel(),
                   split_bytes={"grad_allreduce": 4 * G, "row_allgather_out": 4 * rows,
                                "row_allgather_in_per_rank": 4 * rows // W},
                   ring_send_bytes_per_rank={"fused": round(2 * (W - 1) / W * 4 * eng.comm.numel()),
                                             "split": round(2 * (W - 1) / W * 4 * G + (W - 1) / W * 4 * rows)})
    del eng, model
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--batch", type=int, default=200)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dataset", default="tgbl-wiki")
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=0,
                    help="events per step over all ranks (strong scaling: BASELINE #4 coin 800 at W 4, #5 comment 600 at W 8)")
    a = ap.parse_args()
    out = [run(W, a.batch, a.steps, a.warmup, a.dataset, a.layers, a.global_batch) for W in a.worlds]
    print(json.dumps({"dp_compute_only": out, "dataset": a.dataset, "layers": a.layers,
                      "note": "rank 0 of a W-rank step on one device, exchange skipped; ring_send_bytes_per_rank = "
                              "the bytes a ring collective sends per rank for the fused all-reduce vs the split "
                              "gradient all-reduce + row all-gather"}))


if __name__ == "__main__":
    main()
