"""GPU tests of the engine's data-parallel slicing, the resident vs per-batch paths, and the
drop-in epoch API end to end."""
import copy
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import PKG

pytestmark = pytest.mark.gpu


def _stream(E=1200, N=350, d=172, seed=2):
    from tgnx.synth import make_stream
    return make_stream("tgbl-wiki", seed=seed, num_events=E, num_nodes=N, msg_dim=d)


def _make(s, world=1, rank=0, max_batch=200, seed=0):
    from tgnx.engine import TgnnEngine
    from tgnx.model import TGNN, getOptimizer
    from tgnx.sampler import LastNeighborLoader
    g = torch.Generator().manual_seed(seed)
    m = TGNN(s.shape.msg_dim, 100, s.shape.num_nodes, "cuda", ring=10, max_batch=max_batch, feat_drop=0.0,
             attn_drop=0.0, generator=g)
    opt = getOptimizer({"gnn": m}, 1e-4)
    ld = LastNeighborLoader(s.shape.num_nodes, 10, device="cuda")
    eng = TgnnEngine(m, ld, torch.from_numpy(s.msg), opt, dst_nodes=torch.from_numpy(s.dst_nodes), seed=7,
                     rank=rank, world=world)
    return m, eng


def test_rank_slices_sum_to_full_batch_gradient():
    from tgnx.data import block_ids
    s = _stream()
    B = 200
    blk = block_ids(s.src, s.dst, B)
    full, e1 = _make(s)
    parts = [_make(s, world=2, rank=r) for r in range(2)]
    rng = np.random.default_rng(0)
    for step in range(3):
        sl = slice(step * B, (step + 1) * B)
        args = (s.src[sl], s.dst[sl], s.t[sl].astype(np.float32), s.msg[sl], blk[sl])
        neg = rng.choice(s.dst_nodes, size=B)
        e1.train_batch(*args, neg=neg, update=False)
        for m, e in parts:
            e.train_batch(*args, neg=neg, update=False)
        torch.cuda.synchronize()
        g = parts[0][0].grad_flat + parts[1][0].grad_flat
        ref = full.grad_flat
        err = (g - ref).abs().max() / ref.abs().max()
        assert float(err) < 1e-5, (step, float(err))
        # the all-reduce result, applied on every rank, gives the same parameters
        for m, e in parts:
            m.grad_flat.copy_(ref)
            e.apply_update(allreduce=False)
        e1.apply_update()
        torch.cuda.synchronize()
        for m, _ in parts:
            assert torch.equal(m.flat, full.flat)
            assert torch.equal(m.time_assoc, full.time_assoc)


def test_resident_and_per_batch_paths_agree(monkeypatch):
    monkeypatch.setenv("TGNX_SYNTH_EVENTS", "4000")
    monkeypatch.setenv("TGNX_EVAL_NEGS", "30")
    from tgnx.data import getDataWithDependecyBlock
    from tgnx.epoch import test, train
    from tgnx.model import getModel, getOptimizer
    from tgnx.neg import NegLinkSamplerDest
    from tgnx.sampler import LastNeighborLoader
    data, tr, va, te, ns, ev, metric = getDataWithDependecyBlock("tgbl-wiki", {"batch_size": 200})
    out = []
    for resident in (True, False):
        g = torch.Generator().manual_seed(0)
        model = getModel(172, 100, data.num_nodes, "cuda", gnn_param={"dim_out": 100, "att_head": 8, "layer": 1},
                         ring=10, max_batch=200, generator=g)
        opt = getOptimizer(model, 1e-4)
        ld = LastNeighborLoader(data.num_nodes, 10, device="cuda")
        nds = NegLinkSamplerDest(torch.unique(data.dst), device="cuda")
        loader = tr if resident else list(iter(tr))
        loss = train(model, data.msg, loader, ld, nds, None, "cuda", opt, torch.nn.BCEWithLogitsLoss())
        ns.reset()
        mrr = test(model, data.msg, va if resident else list(iter(va)), ld, ns, None, "cuda", opt, None, ev,
                   metric, "val")
        out.append((loss, mrr, model["gnn"].flat.clone(), ld.e_id.clone()))
    (l0, m0, p0, r0), (l1, m1, p1, r1) = out
    assert np.isfinite(l0) and 0.0 < m0 <= 1.0
    assert abs(l0 - l1) < 1e-6 * abs(l0) and abs(m0 - m1) < 1e-9
    assert torch.equal(p0, p1) and torch.equal(r0, r1)


def test_entry_script_runs_one_epoch():
    env = dict(os.environ, TGNX_SYNTH_EVENTS="6000", TGNX_EVAL_NEGS="50")
    r = subprocess.run([sys.executable, os.path.join(PKG, "pyg-mem-tgn.py"), "--data", "tgbl-wiki",
                        "--epochs", "2", "--batch", "200"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Validation mrr" in r.stdout and "ap and auc" in r.stdout, r.stdout[-2000:]


def test_folded_cursor_equals_advance_plus_step():
    """tgnx_tgnn_train_step_resident (the batch cursor folded into tgnn_assemble, the counter advanced in the next
    launch; the gradient expansion + Adam deferred into the next step's first launch, applied here by finish()) and tgnx_tgnn_train_fwd_bwd_resident + the
    separate update, against tgnx_tgnn_advance + tgnx_tgnn_train_fwd_bwd + tgnx_tgnn_train_update: the same
    parameters, Adam moments, gradients, ring, time_assoc, outputs and every ctl word after each replayed step of a
    split whose last batch is partial, then a step past the split, with device-drawn negatives and dropout."""
    from tgnx.data import block_ids
    s = _stream(E=1300)
    B = 200
    blk = torch.from_numpy(block_ids(s.src, s.dst, B)).cuda()
    dev = torch.device("cuda")
    ev = [torch.from_numpy(x).to(dev) for x in (s.src, s.dst, s.t.astype(np.float32))]
    msg = torch.from_numpy(s.msg).to(dev)
    engs = []
    for fold, fuse in ((True, True), (True, False), (False, False)):
        m, e = _make(s)
        m.cfg.feat_drop = m.cfg.attn_drop = 0.6
        e.fold_cursor, e.fuse_adam = fold, fuse
        neg_buf = torch.zeros(s.num_events, dtype=torch.long, device=dev)
        e.bind_resident(ev[0], ev[1], ev[2], blk, msg, neg_buf, 0, 1100, B, dropout=True)
        assert e._fold == fold and e._fused == fuse
        e.begin_epoch()
        e.capture_resident(1)
        engs.append((m, e, neg_buf))
    for st in range(7):      # 5 full batches, a partial one (100 events), one past the split
        for m, e, _ in engs:
            e.replay_resident()
            e.finish()           # (the deferred-update engine: apply the step's update before comparing)
        torch.cuda.synchronize()
        ma, ea, na = engs[-1]
        ea.check()
        for mb, eb, nb in engs[:-1]:
            eb.check()
            assert torch.equal(ea.ctl, eb.ctl), (st, ea.ctl.tolist(), eb.ctl.tolist())
            assert torch.equal(ma.flat, mb.flat) and torch.equal(ma.time_assoc, mb.time_assoc), st
            assert torch.equal(ea.adam_m, eb.adam_m) and torch.equal(ea.adam_v, eb.adam_v), st
            if st < 6:   # past the split no step runs: the gradient buffer is stale, not part of the state
                assert torch.equal(ma.grad_flat[:-1], mb.grad_flat[:-1]), st
            assert torch.equal(ea.loader.e_id, eb.loader.e_id) and torch.equal(na, nb), st
            assert torch.equal(ea.out_pos, eb.out_pos) and torch.equal(ea.out_neg, eb.out_neg), st


def test_deferred_update_is_applied_before_eval():
    """The world-1 resident step leaves its update pending (applied by the next step's first launch); an eval step
    run right after — no finish() — applies it first: the same logits and parameters as the separate update."""
    from tgnx.data import block_ids
    s = _stream(E=1300)
    B = 200
    blk = torch.from_numpy(block_ids(s.src, s.dst, B)).cuda()
    dev = torch.device("cuda")
    ev = [torch.from_numpy(x).to(dev) for x in (s.src, s.dst, s.t.astype(np.float32))]
    msg = torch.from_numpy(s.msg).to(dev)
    engs = []
    for fuse in (True, False):
        m, e = _make(s)
        e.fuse_adam = fuse
        neg_buf = torch.zeros(s.num_events, dtype=torch.long, device=dev)
        e.bind_resident(ev[0], ev[1], ev[2], blk, msg, neg_buf, 0, 1000, B, dropout=False)
        assert e._defer == fuse
        e.begin_epoch()
        e.capture_resident(1)
        for _ in range(3):
            e.replay_resident()
        engs.append((m, e))
    (ma, ea), (mb, eb) = engs
    torch.cuda.synchronize()
    assert int(ea.ctl[17]) == 3 and not torch.equal(ma.flat, mb.flat)   # step 3's update pending in the first
    sl = slice(1000, 1000 + B)
    neg2d = np.random.default_rng(5).choice(s.dst_nodes, size=(B, 1))   # (the engines' max_neg)
    outs = []
    for m, e in engs:
        e.loader.cur_e_id = 1000
        pos, neg, _ = e.eval_batch(s.src[sl], s.dst[sl], s.t[sl].astype(np.float32), s.msg[sl], block_ids(s.src[sl], s.dst[sl], B), neg2d)
        outs.append((pos.clone(), neg.clone()))
    torch.cuda.synchronize()
    assert int(ea.ctl[17]) == 0
    assert torch.equal(ma.flat, mb.flat) and torch.equal(ea.adam_m, eb.adam_m) and torch.equal(ea.adam_v, eb.adam_v)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_grouped_replay_equals_per_step_replay():
    """World 1: k resident steps captured as one graph (TgnnEngine.capture_group / replay_resident_n, what bench.py's
    timed window replays) against one graph per step — bit-identical state (the TGNN step is deterministic)."""
    from tgnx.data import block_ids
    s = _stream(E=4000)
    B = 200
    blk = torch.from_numpy(block_ids(s.src, s.dst, B)).cuda()
    dev = torch.device("cuda")
    ev = [torch.from_numpy(x).to(dev) for x in (s.src, s.dst, s.t.astype(np.float32))]
    msg = torch.from_numpy(s.msg).to(dev)
    engs = []
    for grouped in (False, True):
        m, e = _make(s)
        m.cfg.feat_drop = m.cfg.attn_drop = 0.6
        neg_buf = torch.zeros(s.num_events, dtype=torch.long, device=dev)
        e.bind_resident(ev[0], ev[1], ev[2], blk, msg, neg_buf, 0, 3800, B, dropout=True)
        e.begin_epoch()
        e.capture_resident(1)
        if grouped:
            assert e.capture_group(8)
        engs.append((m, e, neg_buf))
    (ma, ea, na), (mb, eb, nb) = engs
    for _ in range(3):
        ea.replay_resident()
        eb.replay_resident()
    for _ in range(16):
        ea.replay_resident()
    eb.replay_resident_n(16)
    for _, e, _ in engs:
        e.finish()
        e.check()
    torch.cuda.synchronize()
    assert torch.equal(ea.ctl, eb.ctl)
    assert torch.equal(ma.flat, mb.flat) and torch.equal(ea.adam_m, eb.adam_m) and torch.equal(ea.adam_v, eb.adam_v)
    assert torch.equal(ma.time_assoc, mb.time_assoc) and torch.equal(ea.loader.e_id, eb.loader.e_id)
    assert torch.equal(na, nb)
