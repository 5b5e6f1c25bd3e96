"""The world-1 parity-set TGN step replayed as 8-step graph groups (TgnEngine.capture_group / replay_resident_n, what
bench.py's timed window runs) against one graph per step (replay_resident), from the same state over 24 steps of a
wiki-shaped stream (timestamps rescaled to 2,000 s, where the trajectory is not chaotic): last_update / ring /
stores exact; memory, parameters, Adam moments and the loss sum within the step's own float-atomic run-to-run drift
(tests/test_gpu_tgn_rccl.py) — measured here between two per-step engines from the same state and allowed 20x, with
floors of 1e-4 absolute (memory), 2e-5 / 1e-3 relative (parameters / moments) and 1e-4 relative (loss).  Over 26 steps
that drift reaches ~2e-4 in memory on some runs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
N, D_MSG, D, B, NB = 9_227, 172, 100, 200, 30


def _engine(s):
    from tgnx.sampler import LastNeighborLoader
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = TGNModel(N, s.num_events, D_MSG, D, dev, ring=10, max_batch=B, max_neg=1, aggr="last", dropout=0.1)
    eng = TgnEngine(model, LastNeighborLoader(N, 10, device=dev),
                    dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg), TgnAdam(model, 1e-3),
                    dst_nodes=s.dst_nodes, seed=7)
    eng.bind_resident(0, NB * B, B, dropout=True)
    eng.begin_epoch()
    eng.capture_resident()
    return eng


def _drift(x, y):
    mx, my = x.model, y.model
    rel = lambda u, v: float((u.double() - v.double()).norm() / (v.double().norm() + 1e-12))
    return (float((mx.memory.memory - my.memory.memory).abs().max()), rel(mx.flat, my.flat), rel(x.adam_m, y.adam_m),
            rel(x.adam_v, y.adam_v), abs(x.loss_sum() - y.loss_sum()) / abs(y.loss_sum()))


def test_grouped_replay_equals_per_step_replay():
    from tgnx.synth import make_stream
    s = make_stream("tgbl-wiki", seed=3, num_events=B * NB)
    span = max(float(s.t[-1] - s.t[0]), 1.0)
    s.t = np.floor((s.t - s.t[0]) * (2000.0 / span))
    a, b, c = _engine(s), _engine(s), _engine(s)      # c: a second per-step engine, the drift reference
    assert b.capture_group(8)
    for e in (a, b, c):    # the same 2 steps first (the first primes the scan sets eagerly)
        e.replay_resident()
        e.replay_resident()
    for _ in range(24):
        a.replay_resident()
        c.replay_resident()
    b.replay_resident_n(24)          # 3 groups of 8
    for e in (a, b, c):
        e.finish()
        e.check()
    torch.cuda.synchronize()
    ma, mb = a.model, b.model
    assert torch.equal(ma.memory.last_update, mb.memory.last_update)
    assert torch.equal(a.loader.e_id, b.loader.e_id) and torch.equal(ma.store, mb.store)
    got, noise = _drift(b, a), _drift(c, a)
    for name, g, n, floor in zip(("memory", "params", "adam_m", "adam_v", "loss"), got, noise,
                                 (1e-4, 2e-5, 1e-3, 1e-3, 1e-4)):
        assert g <= max(floor, 20 * n), (name, g, n)
