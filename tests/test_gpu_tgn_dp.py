"""GPU test of the TGN memory path's data-parallel mode (tgnx_tgn_train_fwd_bwd with ctl
rank / world, tgnx_tgn_apply_rows) on one device: two rank engines (world = 2) each run their event
slice of the same global batches; the host sums their gradients (the all-reduce) and concatenates
their packed memory rows (the all-gather); both apply them.  Compared against a world = 1 engine
on the same batches, with device-drawn negatives and attention dropout ON (both keyed so that
they do not depend on the rank or on batch-local numbering).  lr = 0 keeps the parameters fixed, so
memory / last_update / outputs / gradients compare step after step (fp tolerance: gradient sums and
the dz atomics differ in order; the time encoding amplifies weight differences by Δt otherwise).
The two ranks must end every step with bit-identical memory tables."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engines(aggr, N=400, B=64, d=16, D=32, nb=8, layers=1):
    from oracle.tgn_ref import RefTGN
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    s = make_stream("tgbl-wiki", seed=9, num_events=B * nb, num_nodes=N, msg_dim=d)
    torch.manual_seed(0)
    sd = RefTGN(N, d, hidden=D, aggr=aggr, dropout=0.1, layers=layers).state_dict()
    dev = torch.device("cuda")
    ev = dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg)
    out = []
    for rank, world in ((0, 1), (0, 2), (1, 2)):
        model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=1, aggr=aggr, dropout=0.1,
                         layers=layers)
        model.load_reference_state(sd)
        opt = TgnAdam(model, 0.0)
        eng = TgnEngine(model, LastNeighborLoader(N, 10, device=dev), ev, opt, dst_nodes=s.dst_nodes, seed=1234,
                        rank=rank, world=world)
        eng.reset_state()
        out.append(eng)
    return s, B, nb, out


@pytest.mark.parametrize("aggr,layers", [("last", 1), ("mean", 1), ("last", 2)])
def test_tgn_data_parallel_matches_single(aggr, layers):
    s, B, nb, (e1, r0, r1) = _engines(aggr, layers=layers)
    PARAM_ORDER = e1.model.param_order
    for st in range(nb):
        a = st * B
        e1.train_batch(a, B, neg=None, dropout=True, update=True)
        for r in (r0, r1):
            r.train_batch(a, B, neg=None, dropout=True, update=False)
        torch.cuda.synchronize()
        for e in (e1, r0, r1):
            e.check()
        # negatives and outputs of each slice
        for rk, r in enumerate((r0, r1)):
            lo, hi = B * rk // 2, B * (rk + 1) // 2
            assert torch.equal(r.neg_train[a + lo:a + hi], e1.neg_train[a + lo:a + hi]), (st, rk)
            assert torch.allclose(r.out_pos[lo:hi], e1.out_pos[lo:hi], atol=1e-5), (st, rk)
            assert torch.allclose(r.out_neg[lo:hi], e1.out_neg[lo:hi], atol=1e-5), (st, rk)
        # all-reduce: the slice gradients sum to the global-batch gradient (+ loss slot)
        gsum = r0.model.grad_flat + r1.model.grad_flat
        g1 = e1.model.grad_flat
        for name in PARAM_ORDER:
            if name.endswith("lin_key.bias"):   # exactly zero gradient, rounding noise only
                continue
            o, n, _ = e1.model._views[name]
            rel = float((gsum[o:o + n] - g1[o:o + n]).norm() / (g1[o:o + n].norm() + 1e-12))
            assert rel < 1e-4, (st, name, rel)
        assert abs(float(gsum[-1]) - float(g1[-1])) < 1e-5
        # all-gather of the packed rows, then every rank applies them
        rows = torch.cat([r0.xrows, r1.xrows])
        for r in (r0, r1):
            r.model.grad_flat.copy_(gsum)
            r.xgather.copy_(rows)
            r.apply_update(allreduce=False)
        torch.cuda.synchronize()
        assert torch.equal(r0.model.memory.memory, r1.model.memory.memory), st
        assert torch.equal(r0.model.memory.last_update, r1.model.memory.last_update), st
        assert torch.equal(r0.model.memory.last_update, e1.model.memory.last_update), st
        assert torch.allclose(r0.model.memory.memory, e1.model.memory.memory, atol=1e-5), \
            (st, float((r0.model.memory.memory - e1.model.memory.memory).abs().max()))
        assert torch.equal(r0.model.store, e1.model.store), st
        assert torch.equal(r0.loader.neighbors, e1.loader.neighbors) and torch.equal(r0.loader.e_id, e1.loader.e_id)


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_tgn_dp_resident_folded_cursor_per_rank():
    """Data-parallel resident steps (world = 2, one device) with the batch cursor folded into the first
    launch (tgnx_tgn_train_fwd_bwd_resident) against tgnx_tgnn_advance + tgnx_tgn_train_fwd_bwd, per rank,
    through the summing exchange, apply_rows and Adam (lr 1e-3, so an ADAM_T off by one shows in the
    parameters): ctl words, the rank's negatives, gradients and packed memory rows after fwd_bwd; memory,
    last_update, parameters and moments after the update.  The split ends with a partial batch (20
    events) and the last step runs one batch past the split (B = 0: nothing may change).  Parameters
    and memory are re-synchronised from the unfolded twin after each compared step (the dz atomics make
    the gradients order-dependent at the last bits)."""
    from oracle.tgn_ref import RefTGN
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    N, B, d, D = 400, 64, 16, 32
    s = make_stream("tgbl-wiki", seed=9, num_events=B * 9, num_nodes=N, msg_dim=d)
    torch.manual_seed(0)
    sd = RefTGN(N, d, hidden=D, aggr="last", dropout=0.1).state_dict()
    dev = torch.device("cuda")
    ev = dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg)
    split_hi = 7 * B + 20
    eng = {}
    for fold in (True, False):
        for rank in (0, 1):
            model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=1, aggr="last", dropout=0.1)
            model.load_reference_state(sd)
            e = TgnEngine(model, LastNeighborLoader(N, 10, device=dev), ev, TgnAdam(model, 1e-3),
                          dst_nodes=s.dst_nodes, seed=77, rank=rank, world=2)
            e.fold_cursor = fold
            e.pipeline = False   # the pipelined forms have their own tests below
            e.bind_resident(0, split_hi, B, dropout=True)
            e.begin_epoch()
            eng[fold, rank] = e
    for st in range(9):
        for e in eng.values():
            e._pre()
        torch.cuda.synchronize()
        for e in eng.values():
            e.check()
        for rank in (0, 1):
            f, u = eng[True, rank], eng[False, rank]
            for w in (0, 1, 2, 3, 4, 7, 8, 9, 10):   # start, cur e_id, B, GEN, ADAM_T, LO, HI, SEED, NB
                assert int(f.ctl[w]) == int(u.ctl[w]), (st, rank, w, int(f.ctl[w]), int(u.ctl[w]))
            Bst = int(u.ctl[2])
            assert Bst == (B if st < 7 else 20 if st == 7 else 0), (st, Bst)
            assert torch.equal(f.neg_train, u.neg_train), (st, rank)
            G = f.model.grad_flat.numel()
            if Bst:
                assert _rel(f.comm[:G - 1], u.comm[:G - 1]) < 1e-5, (st, rank)
                assert abs(float(f.comm[G - 1]) - float(u.comm[G - 1])) < 1e-5, (st, rank)
            assert torch.equal(f.xrows, u.xrows), (st, rank)  # node headers and GRU rows (deterministic GEMM)
        # the exchange (all-reduce = sum over ranks), per twin set
        for fold in (True, False):
            tot = eng[fold, 0].comm + eng[fold, 1].comm
            for rank in (0, 1):
                eng[fold, rank].comm.copy_(tot)
        for e in eng.values():
            e._post()
        torch.cuda.synchronize()
        for rank in (0, 1):
            f, u = eng[True, rank], eng[False, rank]
            fm, um = f.model, u.model
            assert torch.equal(fm.memory.last_update, um.memory.last_update), (st, rank)
            assert torch.allclose(fm.memory.memory, um.memory.memory, atol=1e-6), (st, rank)
            assert _rel(fm.flat, um.flat) < 1e-6, (st, rank)
            assert _rel(f.adam_m, u.adam_m) < 1e-5 and _rel(f.adam_v, u.adam_v) < 1e-5, (st, rank)
            assert abs(f.loss_sum() - u.loss_sum()) <= 1e-6 * max(1.0, abs(u.loss_sum())), (st, rank)
            assert torch.equal(f.loader.e_id, u.loader.e_id) and torch.equal(f.model.store, u.model.store), (st, rank)
        assert torch.equal(eng[True, 0].model.memory.memory, eng[True, 1].model.memory.memory), st
        for rank in (0, 1):   # re-synchronise the folded twin
            f, u = eng[True, rank], eng[False, rank]
            with torch.no_grad():
                f.model.flat.copy_(u.model.flat)
                f.adam_m.copy_(u.adam_m)
                f.adam_v.copy_(u.adam_v)
                f.model.memory.memory.copy_(u.model.memory.memory)


@pytest.mark.parametrize("split", [True, False])
def test_tgn_dp_pipelined_per_rank(split):
    """Data-parallel pipelined steps (tgnx_tgn_train_fwd_bwd_pipelined, world = 2, one device: each step
    marks its rank's slice of the NEXT batch in the k / v reduction launch and scans it after its last
    launch; tgnx_tgn_apply_rows_update writes the exchanged rows and runs Adam in one launch) against the
    folded resident steps + apply_rows + train_update, per rank: counters, negatives, gradients and packed
    rows after fwd_bwd; memory, last_update, parameters, moments and loss after the update.  The split ends
    with a partial batch (20 events) and one step runs past it (B = 0: memory — node 0 included — and
    parameters must not change).  The pipelined twin is re-synchronised from the folded one after each step."""
    from oracle.tgn_ref import RefTGN
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    N, B, d, D = 400, 64, 16, 32
    s = make_stream("tgbl-wiki", seed=9, num_events=B * 9, num_nodes=N, msg_dim=d)
    torch.manual_seed(0)
    sd = RefTGN(N, d, hidden=D, aggr="last", dropout=0.1).state_dict()
    dev = torch.device("cuda")
    ev = dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg)
    split_hi = 7 * B + 20
    eng = {}
    for pipe in (True, False):
        for rank in (0, 1):
            model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=1, aggr="last", dropout=0.1)
            model.load_reference_state(sd)
            e = TgnEngine(model, LastNeighborLoader(N, 10, device=dev), ev, TgnAdam(model, 1e-3),
                          dst_nodes=s.dst_nodes, seed=77, rank=rank, world=2)
            e.pipeline = pipe
            e.parity_sets = False  # (the parity-set step: test_tgn_dp_parity_sets_per_rank)
            e.split_scan = split   # the next batch's scan beside the exchange (tgnx_tgn_scan_next) or in fwd_bwd
            e.bind_resident(0, split_hi, B, dropout=True)
            e.begin_epoch()
            assert e._pipelined() == pipe and e._split() == (pipe and split)
            eng[pipe, rank] = e
    for st in range(9):
        mem0 = eng[False, 0].model.memory.memory.clone()
        flat0 = eng[False, 0].model.flat.clone()
        for e in eng.values():
            e._pre(e._prefetched)
        torch.cuda.synchronize()
        for e in eng.values():
            e.check()
        end = min(split_hi, (st + 1) * B)
        for rank in (0, 1):
            p, u = eng[True, rank], eng[False, rank]
            for w in (3, 4, 10, 16):   # GEN, ADAM_T, NB, STEP_B
                assert int(p.ctl[w]) == int(u.ctl[w]), (st, rank, w, int(p.ctl[w]), int(u.ctl[w]))
            Bst = int(u.ctl[16])
            assert Bst == (B if st < 7 else 20 if st == 7 else 0), (st, Bst)
            assert torch.equal(p.neg_train[:end], u.neg_train[:end]), (st, rank)
            G = p.model.grad_flat.numel()
            if Bst:
                assert _rel(p.comm[:G - 1], u.comm[:G - 1]) < 1e-5, (st, rank)
                assert abs(float(p.comm[G - 1]) - float(u.comm[G - 1])) < 1e-5, (st, rank)
            assert torch.equal(p.xrows, u.xrows), (st, rank)
        for pipe in (True, False):
            tot = eng[pipe, 0].comm + eng[pipe, 1].comm
            for rank in (0, 1):
                eng[pipe, rank].comm.copy_(tot)
        for e in eng.values():
            e._scan_next()   # (split: the next batch's scan, which rides beside the exchange)
            e._post()
            e._prefetched = e._pipelined()
        torch.cuda.synchronize()
        for rank in (0, 1):
            p, u = eng[True, rank], eng[False, rank]
            pm, um = p.model, u.model
            assert torch.equal(pm.memory.last_update, um.memory.last_update), (st, rank)
            assert torch.allclose(pm.memory.memory, um.memory.memory, atol=1e-6), (st, rank)
            assert _rel(pm.flat, um.flat) < 1e-6, (st, rank)
            assert _rel(p.adam_m, u.adam_m) < 1e-5 and _rel(p.adam_v, u.adam_v) < 1e-5, (st, rank)
            assert abs(p.loss_sum() - u.loss_sum()) <= 1e-6 * max(1.0, abs(u.loss_sum())), (st, rank)
            assert torch.equal(p.loader.e_id, u.loader.e_id) and torch.equal(p.model.store, u.model.store), (st, rank)
        if st == 8:   # past the split: nothing changes (the exchange slots read as unused, Adam skips)
            for e in eng.values():
                assert torch.equal(e.model.memory.memory, mem0), st
                assert torch.equal(e.model.flat, flat0), st
        assert torch.equal(eng[True, 0].model.memory.memory, eng[True, 1].model.memory.memory), st
        for rank in (0, 1):
            p, u = eng[True, rank], eng[False, rank]
            with torch.no_grad():
                p.model.flat.copy_(u.model.flat)
                p.adam_m.copy_(u.adam_m)
                p.adam_v.copy_(u.adam_v)
                p.model.memory.memory.copy_(u.model.memory.memory)


@pytest.mark.parametrize("graphs,layers", [(True, 1), (False, 1), (True, 2), (False, 2)])
def test_tgn_dp_parity_sets_per_rank(graphs, layers):
    """The data-parallel parity-set step (tgnx_tgn_train_fwd_bwd_pp, world = 2, one device: the next batch's
    slice marked in the predictor launch and scanned into the other parity set inside the dW_cell launch; the
    exchanged rows + Adam of step k at the head of step k + 1) against the split pipelined step
    (tgnx_tgn_train_fwd_bwd_split + tgnx_tgn_scan_next + tgnx_tgn_apply_rows_update), per rank, lr 1e-3.
    The parity-set engines run through the engine's own step (graph replays or eager steps) with the
    collective replaced by a no-op; the test sums the exchange buffers of both ranks between steps, then
    finish() applies them (so the next replay takes the graph without the apply at its head).  Per step:
    counters, negatives, gradients + loss slot and packed rows before the apply; memory, last_update,
    parameters, moments, loss sum, ring and stores after it.  A partial batch and one step past the split.
    layers = 2: the 2-hop parity-set step (the root level's scan outputs doubled, plan table), what BASELINE
    config #5 runs at world 8, against the 2-hop split step."""
    from oracle.tgn_ref import RefTGN
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    N, B, d, D = 400, 64, 16, 32
    s = make_stream("tgbl-wiki", seed=9, num_events=B * 9, num_nodes=N, msg_dim=d)
    torch.manual_seed(0)
    sd = RefTGN(N, d, hidden=D, aggr="last", dropout=0.1, layers=layers).state_dict()
    dev = torch.device("cuda")
    ev = dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg)
    split_hi = 7 * B + 20
    eng = {}
    for pp in (True, False):
        for rank in (0, 1):
            model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=1, aggr="last", dropout=0.1,
                             layers=layers)
            model.load_reference_state(sd)
            e = TgnEngine(model, LastNeighborLoader(N, 10, device=dev), ev, TgnAdam(model, 1e-3),
                          dst_nodes=s.dst_nodes, seed=77, rank=rank, world=2)
            e.parity_sets = pp
            e.exchange = lambda comm, async_op: None
            e.bind_resident(0, split_hi, B, dropout=True)
            e.begin_epoch()
            assert e._dp_pp() == pp and e._split() == (not pp)
            if pp and graphs:
                e.capture_resident()
            eng[pp, rank] = e
    for st in range(9):
        for rank in (0, 1):
            p = eng[True, rank]
            if graphs:
                p.replay_resident()
            else:
                p.resident_train_step()
            u = eng[False, rank]
            u._pre(u._prefetched)
        torch.cuda.synchronize()
        for e in eng.values():
            e.check(settle=False)   # (the test sums the exchange itself below)
        end = min(split_hi, (st + 1) * B)
        for rank in (0, 1):
            p, u = eng[True, rank], eng[False, rank]
            for w in (3, 4, 10, 16):   # GEN, ADAM_T, NB, STEP_B
                assert int(p.ctl[w]) == int(u.ctl[w]), (st, rank, w, int(p.ctl[w]), int(u.ctl[w]))
            Bst = int(u.ctl[16])
            assert Bst == (B if st < 7 else 20 if st == 7 else 0), (st, Bst)
            assert torch.equal(p.neg_train[:end], u.neg_train[:end]), (st, rank)
            G = p.model.grad_flat.numel()
            if Bst:
                assert _rel(p.comm[:G - 1], u.comm[:G - 1]) < 1e-5, (st, rank)
                assert abs(float(p.comm[G - 1]) - float(u.comm[G - 1])) < 1e-5, (st, rank)
                lo, hi = Bst * rank // 2, Bst * (rank + 1) // 2
                assert torch.allclose(p.out_pos[lo:hi], u.out_pos[lo:hi], atol=1e-6), (st, rank)
            assert torch.equal(p.xrows, u.xrows), (st, rank)
        for pp in (True, False):
            tot = eng[pp, 0].comm + eng[pp, 1].comm
            for rank in (0, 1):
                eng[pp, rank].comm.copy_(tot)
        for rank in (0, 1):
            p, u = eng[True, rank], eng[False, rank]
            assert p._apply_pending
            p.finish()
            u._scan_next()
            u._post()
            u._prefetched = True
        torch.cuda.synchronize()
        for rank in (0, 1):
            p, u = eng[True, rank], eng[False, rank]
            pm, um = p.model, u.model
            for w in (0, 1, 2, 7, 8, 9, 11):   # the next batch's descriptor (both prefetched it), no error
                assert int(p.ctl[w]) == int(u.ctl[w]), (st, rank, w)
            assert torch.equal(pm.memory.last_update, um.memory.last_update), (st, rank)
            assert torch.allclose(pm.memory.memory, um.memory.memory, atol=1e-6), (st, rank)
            assert _rel(pm.flat, um.flat) < 1e-6, (st, rank)
            assert _rel(p.adam_m, u.adam_m) < 1e-5 and _rel(p.adam_v, u.adam_v) < 1e-5, (st, rank)
            assert abs(p.loss_sum() - u.loss_sum()) <= 1e-6 * max(1.0, abs(u.loss_sum())), (st, rank)
            assert torch.equal(p.loader.e_id, u.loader.e_id) and torch.equal(p.model.store, u.model.store), (st, rank)
            assert torch.equal(p.xgather, torch.zeros_like(p.xgather)), (st, rank)   # slots zeroed by the apply
        assert torch.equal(eng[True, 0].model.memory.memory, eng[True, 1].model.memory.memory), st
        for rank in (0, 1):   # re-synchronise the parity-set twin
            p, u = eng[True, rank], eng[False, rank]
            with torch.no_grad():
                p.model.flat.copy_(u.model.flat)
                p.adam_m.copy_(u.adam_m)
                p.adam_v.copy_(u.adam_v)
                p.model.memory.memory.copy_(u.model.memory.memory)
