"""GPU parity of the TGN memory path (SURVEY §8 a14–a16, tgnx_tgn_*) against the oracle restatement
oracle/tgn_ref.py (PARITY UNPINNED for its torch_geometric / torch_scatter parts, see its header).

Step by step on a small wiki-shaped stream with injected negatives and dropout off: link-prediction
outputs, every parameter gradient, the TGNMemory state (memory, last_update) after update_state, the
parameters after Adam; then flush (train(False)) and TGB-style eval scores / reciprocal ranks.
Parameters, Adam moments and memory are resynchronised from the oracle after each compared step
(fp32 reduction order differs; the comparison is per step).  Tolerances: outputs 2e-5 abs, memory
1e-5 abs, gradients 2e-3 relative (L2) per tensor.  gnn.conv.lin_key.bias has an exactly zero
gradient (q_i·b_k is the same for every edge of a centre, softmax is shift invariant): both sides
hold rounding noise, checked to be negligible against lin_key.weight's gradient, and Adam turns that
noise into lr-sized steps, so its parameters are excluded from the after-step comparison."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHIFT_INVARIANT = {"gnn.conv.lin_key.bias": "gnn.conv.lin_key.weight", "gnn.conv2.lin_key.bias": "gnn.conv2.lin_key.weight"}


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _setup(aggr, N=300, B=50, d=16, D=32, nb=10, seed=3, max_neg=20, layers=1, updater="gru", memory="tgn", emb=(0, 0)):
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    s = make_stream("tgbl-wiki", seed=seed, num_events=B * nb, num_nodes=N, msg_dim=d)
    torch.manual_seed(0)
    ref = RefTGN(N, d, hidden=D, aggr=aggr, dropout=0.0, layers=layers, updater=updater,
                 use_src_emb_in_msg=bool(emb[0]), use_dst_emb_in_msg=bool(emb[1]))
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    dev = torch.device("cuda")
    model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=max_neg, aggr=aggr, dropout=0.0,
                     layers=layers, updater=updater, memory=memory, use_src_emb_in_msg=bool(emb[0]),
                     use_dst_emb_in_msg=bool(emb[1]))
    model.load_reference_state(ref.state_dict())
    opt = TgnAdam(model, 1e-3)
    loader = LastNeighborLoader(N, 10, device=dev)
    eng = TgnEngine(model, loader, dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg), opt,
                    dst_nodes=s.dst_nodes)
    eng.reset_state()
    return s, ref, opt_ref, RefLastNeighborLoader(N, 10), model, opt, eng


def _sync(ref, opt_ref, model, opt):
    named = dict(ref.named_parameters())
    with torch.no_grad():
        for name in model.param_order:
            o, n, _ = model._views[name]
            p = named[name]
            model.flat[o:o + n].copy_(p.detach().reshape(-1))
            st = opt_ref.state.get(p, {})
            if st:
                opt.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                opt.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
        model.memory.memory.copy_(ref.memory.memory)
        model.memory.last_update.copy_(ref.memory.last_update)


@pytest.mark.parametrize("aggr,layers,updater,emb", [("last", 1, "gru", (0, 0)), ("mean", 1, "gru", (0, 0)),
                                                      ("last", 2, "gru", (0, 0)), ("mean", 2, "gru", (0, 0)),
                                                      ("last", 1, "rnn", (0, 0)), ("mean", 1, "rnn", (0, 0)),
                                                      ("last", 2, "rnn", (0, 0)), ("last", 1, "rnn", (1, 1)),
                                                      ("mean", 1, "rnn", (0, 1)), ("last", 1, "gru", (1, 0))])
def test_tgn_train_steps_and_eval_match_oracle(aggr, layers, updater, emb):
    """layers = 2: the 2-hop extension (oracle RefTGN(layers=2); no reference parity possible).
    updater = 'rnn': the RNNCell memory updater (TGNMemory memory_updater_cell / DyRepMemory
    memory_updater_type, memory_module.py:70-78, :259-264; the engine built as DyRepMemory).
    emb: DyRepMemory (use_src_emb_in_msg, use_dst_emb_in_msg) (memory_module.py:387-408): update_state's
    messages carry the batch's embeddings for endpoints in src ∪ dst (train and eval forwards)."""
    from oracle.tgn_ref import eval_step, mrr_per_event, train_step
    B = 50
    s, ref, opt_ref, lref, model, opt, eng = _setup(aggr, layers=layers, updater=updater,
                                                    memory="dyrep" if updater == "rnn" or any(emb) else "tgn",
                                                    emb=emb)
    PARAM_ORDER = model.param_order
    ev_t = torch.from_numpy(s.t.astype(np.float32))
    ev_msg = torch.from_numpy(s.msg)
    rng = np.random.default_rng(1)
    named = dict(ref.named_parameters())
    worst = {}
    for st in range(7):
        a = st * B
        sl = slice(a, a + B)
        src, pos = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
        neg = torch.from_numpy(rng.choice(s.dst_nodes, size=B))
        loss, po, no = train_step(ref, opt_ref, lref, ev_t, ev_msg, src, pos, neg, ev_t[sl], ev_msg[sl])
        pg, ng = eng.train_batch(a, B, neg=neg)
        torch.cuda.synchronize()
        eng.check()
        assert torch.allclose(pg.cpu(), po, atol=2e-5), (st, (pg.cpu() - po).abs().max())
        assert torch.allclose(ng.cpu(), no, atol=2e-5), (st, (ng.cpu() - no).abs().max())
        assert abs(float(model.grad_flat[-1]) - loss) < 1e-5 * max(1.0, abs(loss))
        g = model.grads_by_name()
        for name in PARAM_ORDER:
            if name in SHIFT_INVARIANT:
                scale = float(named[SHIFT_INVARIANT[name]].grad.norm()) + 1e-12
                assert float(g[name].norm()) < 1e-4 * scale and float(named[name].grad.norm()) < 1e-4 * scale
                continue
            r = _rel(g[name], named[name].grad)
            worst[name] = max(worst.get(name, 0.0), r)
            assert r < 2e-3, (st, name, r)
        assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5), st
        assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update), st
        for name in PARAM_ORDER:
            if name in SHIFT_INVARIANT:
                continue
            o, n, _ = model._views[name]
            assert torch.allclose(model.flat[o:o + n].cpu(), named[name].detach().reshape(-1), atol=5e-6, rtol=1e-4), \
                (st, name)
        _sync(ref, opt_ref, model, opt)
    # train(False): flush both, then a TGB-style eval batch
    ref.memory.train(False)
    eng.flush()
    torch.cuda.synchronize()
    assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5)
    assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update)
    a = 7 * B
    sl = slice(a, a + B)
    src, pos = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
    negs = torch.from_numpy(rng.choice(s.dst_nodes, size=(B, 20)))
    po, no = eval_step(ref, lref, ev_t, ev_msg, src, pos, negs, ev_t[sl], ev_msg[sl])
    pg, ngm, rr = eng.eval_batch(a, B, negs)
    torch.cuda.synchronize()
    eng.check()
    assert torch.allclose(pg.cpu(), po, atol=2e-5)
    assert torch.allclose(ngm.cpu(), no, atol=2e-5)
    # reciprocal ranks: exact unless a negative ties the positive within the score tolerance
    close = ((no - po.view(-1, 1)).abs() <= 4e-5).any(1).numpy()
    assert np.allclose(rr.cpu().numpy()[~close], mrr_per_event(po, no)[~close], atol=1e-6)
    assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5)
    assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update)


@pytest.mark.parametrize("layers", [1, 2])
def test_tgn_fused_adam_step_equals_fwd_bwd_plus_update(layers):
    """tgnx_tgn_train_step (Adam folded into the gradient writers) against tgnx_tgn_train_fwd_bwd +
    tgnx_tgn_train_update on twin engines, device negatives and attention dropout on.  The gradient
    atomics (dz rows, neighbour k/v sums) make the two runs' gradients differ in the last bits, so
    the states are resynchronised after every step and compared per step: outputs 1e-5 abs;
    parameters and Adam moments per tensor 1e-4 relative (the shift-invariant lin_key.bias, whose
    gradient is pure rounding noise, excluded); memory 1e-5 abs; loss sums 1e-5 relative."""
    engines = []
    for fused in (True, False):
        s, ref, opt_ref, lref, model, opt, eng = _setup("last", layers=layers)
        model.cfg.dropout = 0.1
        eng.fuse_adam = fused
        engines.append((model, opt, eng))
    (m1, o1, e1), (m2, o2, e2) = engines
    B = 50
    for st in range(6):
        outs = [e.train_batch(st * B, B, neg=None, dropout=True, update=True) for e in (e1, e2)]
        torch.cuda.synchronize()
        e1.check()
        e2.check()
        assert torch.allclose(outs[0][0], outs[1][0], atol=1e-5) and torch.allclose(outs[0][1], outs[1][1], atol=1e-5)
        for name in m1.param_order:
            if name in SHIFT_INVARIANT:
                continue
            o, n, _ = m1._views[name]
            for a, b in ((m1.flat, m2.flat), (o1.exp_avg, o2.exp_avg), (o1.exp_avg_sq, o2.exp_avg_sq)):
                assert _rel(a[o:o + n], b[o:o + n]) < 1e-4, (st, name)
        assert torch.allclose(m1.memory.memory, m2.memory.memory, atol=1e-5), st
        assert abs(e1.loss_sum() - e2.loss_sum()) <= 1e-5 * abs(e2.loss_sum()), st
        with torch.no_grad():   # resynchronise: the next step starts from identical states
            m1.flat.copy_(m2.flat)
            o1.exp_avg.copy_(o2.exp_avg)
            o1.exp_avg_sq.copy_(o2.exp_avg_sq)
            m1.memory.memory.copy_(m2.memory.memory)


def test_tgn_mean_hub_node_matches_oracle():
    """MeanAggregator over a hub: one node is the source of EVERY event of a 300-event batch, so in the
    next batch its stored messages (300) are split over the four waves of its workgroup, each wave
    running more than one 64-message round (agg_node_mean_wg), in the train step and in the eval
    update.  Outputs, gradients, memory and last_update against the oracle as in the main test."""
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, eval_step, train_step
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    N, B, d, D, nb = 400, 300, 8, 32, 4
    s = make_stream("tgbl-wiki", seed=5, num_events=B * nb, num_nodes=N, msg_dim=d)
    hub = int(s.src[0])
    s.src[:] = hub                      # the hub is every event's source
    torch.manual_seed(0)
    ref = RefTGN(N, d, hidden=D, aggr="mean", dropout=0.0)
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    dev = torch.device("cuda")
    model = TGNModel(N, s.num_events, d, D, dev, ring=10, max_batch=B, max_neg=5, aggr="mean", dropout=0.0)
    model.load_reference_state(ref.state_dict())
    opt = TgnAdam(model, 1e-3)
    eng = TgnEngine(model, LastNeighborLoader(N, 10, device=dev),
                    dict(src=s.src, dst=s.dst, t=s.t.astype(np.float32), msg=s.msg), opt, dst_nodes=s.dst_nodes)
    eng.reset_state()
    lref = RefLastNeighborLoader(N, 10)
    ev_t, ev_msg = torch.from_numpy(s.t.astype(np.float32)), torch.from_numpy(s.msg)
    rng = np.random.default_rng(2)
    named = dict(ref.named_parameters())
    for st in range(nb - 1):
        sl = slice(st * B, (st + 1) * B)
        src, pos = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
        neg = torch.from_numpy(rng.choice(s.dst_nodes, size=B))
        loss, po, no = train_step(ref, opt_ref, lref, ev_t, ev_msg, src, pos, neg, ev_t[sl], ev_msg[sl])
        pg, ng = eng.train_batch(st * B, B, neg=neg)
        torch.cuda.synchronize()
        eng.check()
        assert torch.allclose(pg.cpu(), po, atol=2e-5) and torch.allclose(ng.cpu(), no, atol=2e-5), st
        g = model.grads_by_name()
        for name in model.param_order:
            if name in SHIFT_INVARIANT:
                continue
            assert _rel(g[name], named[name].grad) < 2e-3, (st, name)
        assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5), st
        assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update), st
        _sync(ref, opt_ref, model, opt)
    # eval batch (scores with the batch-start state, then the eval update aggregates the hub again)
    ref.memory.train(False)
    eng.flush()
    a = (nb - 1) * B
    sl = slice(a, a + B)
    src, pos = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
    negs = torch.from_numpy(rng.choice(s.dst_nodes, size=(B, 5)))
    po, no = eval_step(ref, lref, ev_t, ev_msg, src, pos, negs, ev_t[sl], ev_msg[sl])
    pg, ngm, rr = eng.eval_batch(a, B, negs)
    torch.cuda.synchronize()
    eng.check()
    assert torch.allclose(pg.cpu(), po, atol=2e-5) and torch.allclose(ngm.cpu(), no, atol=2e-5)
    assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5)
    assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update)


def test_tgn_resident_folded_cursor_equals_advance_plus_step():
    """Resident world-1 steps with the batch cursor folded into tgn_mark (tgnx_tgn_train_step_resident)
    against tgnx_tgnn_advance + tgnx_tgn_train_step on a twin engine, device negatives and attention
    dropout on: the step counters and batch descriptor in ctl must match exactly after every step;
    outputs, parameters and memory within the fused-Adam test's tolerances (resynchronised per step)."""
    engines = []
    for fold in (True, False):
        s, ref, opt_ref, lref, model, opt, eng = _setup("last")
        model.cfg.dropout = 0.1
        eng.fold_cursor = fold
        eng.pipeline = False
        eng.bind_resident(0, 7 * 50 + 20, 50, dropout=True)   # the last batch is partial (20 events)
        eng.begin_epoch()
        engines.append((model, opt, eng))
    (m1, o1, e1), (m2, o2, e2) = engines
    for st in range(9):                                        # 8 batches, then one past the split (B = 0)
        for e in (e1, e2):
            e.resident_train_step()
        torch.cuda.synchronize()
        e1.check()
        e2.check()
        for w in (0, 1, 2, 3, 4, 7, 8, 9, 10):                 # start, cur e_id, B, GEN, ADAM_T, LO, HI, SEED, NB
            assert int(e1.ctl[w]) == int(e2.ctl[w]), (st, w, int(e1.ctl[w]), int(e2.ctl[w]))
        assert torch.equal(e1.neg_train, e2.neg_train), st
        B = int(e1.ctl[2])
        if B:
            assert torch.allclose(e1.out_pos[:B], e2.out_pos[:B], atol=1e-5), st
        for name in m1.param_order:
            if name in SHIFT_INVARIANT:
                continue
            o, n, _ = m1._views[name]
            assert _rel(m1.flat[o:o + n], m2.flat[o:o + n]) < 1e-4, (st, name)
        assert torch.allclose(m1.memory.memory, m2.memory.memory, atol=1e-5), st
        assert abs(e1.loss_sum() - e2.loss_sum()) <= 1e-5 * max(1.0, abs(e2.loss_sum())), st
        with torch.no_grad():
            m1.flat.copy_(m2.flat)
            o1.exp_avg.copy_(o2.exp_avg)
            o1.exp_avg_sq.copy_(o2.exp_avg_sq)
            m1.memory.memory.copy_(m2.memory.memory)


@pytest.mark.parametrize("pp,table", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("layers,updater,emb", [(1, "gru", (0, 0)), (2, "gru", (0, 0)), (1, "rnn", (0, 0)),
                                                (1, "rnn", (1, 1))])
def test_tgn_pipelined_equals_resident(layers, updater, emb, pp, table):
    """tgnx_tgn_train_step_pipelined (each step marks the next batch inside its predictor launch and scans it
    after its last launch; ring insert beside the GRU) — or, pp (1 or 2 hops), tgnx_tgn_train_step_pp (the next
    batch scanned into the other parity's set inside an earlier launch of the step, two graphs replayed alternately) —
    against tgnx_tgn_train_step_resident on a twin engine: graph replay (the first step eager with
    prefetched = 0), device negatives, attention dropout, a partial last batch and a step past the split.
    After every step: step counters and the ring exactly, this batch's negatives exactly (the pipelined
    engine has drawn the next batch's too), outputs, parameters and memory within the fused-Adam tolerances
    (resynchronised per step).  table: the parity-set step reads the split's plans from the table built at
    binding (tgnx_tgn_plan_table) instead of its scan's, which then only walks the node sets."""
    engines = []
    for pipe in (True, False):
        s, ref, opt_ref, lref, model, opt, eng = _setup("last", layers=layers, updater=updater,
                                                        memory="dyrep" if any(emb) else "tgn", emb=emb)
        model.cfg.dropout = 0.1
        eng.pipeline = pipe
        eng.parity_sets = pp
        eng.use_plan_table = table and pipe
        eng.bind_resident(0, 7 * 50 + 20, 50, dropout=True)   # the last batch is partial (20 events)
        eng.begin_epoch()
        if pipe:
            eng.capture_resident()
        engines.append((model, opt, eng))
    (m1, o1, e1), (m2, o2, e2) = engines
    for st in range(9):                                        # 8 batches, then one past the split (B = 0)
        e1.replay_resident()
        e2.resident_train_step()
        torch.cuda.synchronize()
        e1.check()
        e2.check()
        for w in (3, 4, 10):                                   # GEN, ADAM_T, NB
            assert int(e1.ctl[w]) == int(e2.ctl[w]), (st, w, int(e1.ctl[w]), int(e2.ctl[w]))
        B, start = int(e2.ctl[2]), int(e2.ctl[0])
        assert torch.equal(e1.neg_train[:start + B], e2.neg_train[:start + B]), st
        for a, b in ((e1.loader.neighbors, e2.loader.neighbors), (e1.loader.e_id, e2.loader.e_id),
                     (e1.loader.t, e2.loader.t)):
            assert torch.equal(a, b), st
        if B:
            assert torch.allclose(e1.out_pos[:B], e2.out_pos[:B], atol=1e-5), st
            assert torch.allclose(e1.out_neg[:B], e2.out_neg[:B], atol=1e-5), st
        for name in m1.param_order:
            if name in SHIFT_INVARIANT:
                continue
            o, n, _ = m1._views[name]
            assert _rel(m1.flat[o:o + n], m2.flat[o:o + n]) < 1e-4, (st, name)
        assert torch.allclose(m1.memory.memory, m2.memory.memory, atol=1e-5), st
        assert torch.equal(m1.memory.last_update, m2.memory.last_update), st
        assert abs(e1.loss_sum() - e2.loss_sum()) <= 1e-5 * max(1.0, abs(e2.loss_sum())), st
        with torch.no_grad():
            m1.flat.copy_(m2.flat)
            o1.exp_avg.copy_(o2.exp_avg)
            o1.exp_avg_sq.copy_(o2.exp_avg_sq)
            m1.memory.memory.copy_(m2.memory.memory)


def test_tgn_large_batch_partitioned_plans_match_oracle():
    """A batch of 1,100 events (2,200 plan keys): the insert and store plans split by node range over
    several workgroups each (plan_part, tgn_scan; P = ceil(2B / 512) = 5), as a data-parallel step plans
    its global batch.  Train steps against the oracle: outputs, memory, last_update, the ring (neighbours,
    e_id, t) and the loader's assoc of the inserted nodes (neighbor_loader.py:72-73: their rank among the
    batch's nodes), then a flush and an eval batch of the same size."""
    from oracle.tgn_ref import train_step
    B, nb = 1100, 3
    s, ref, opt_ref, lref, model, opt, eng = _setup("last", N=3000, B=B, nb=nb + 1, max_neg=1)
    ev_t = torch.from_numpy(s.t.astype(np.float32))
    ev_msg = torch.from_numpy(s.msg)
    rng = np.random.default_rng(5)
    for st in range(nb):
        a = st * B
        sl = slice(a, a + B)
        src, pos = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
        neg = torch.from_numpy(rng.choice(s.dst_nodes, size=B))
        _, po, no = train_step(ref, opt_ref, lref, ev_t, ev_msg, src, pos, neg, ev_t[sl], ev_msg[sl])
        pg, ng = eng.train_batch(a, B, neg=neg)
        torch.cuda.synchronize()
        eng.check()
        assert torch.allclose(pg.cpu(), po, atol=2e-5) and torch.allclose(ng.cpu(), no, atol=2e-5), st
        assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5), st
        assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update), st
        assert np.array_equal(eng.loader.e_id.cpu().numpy(), lref.e_id), st
        live = lref.e_id >= 0
        assert np.array_equal(eng.loader.neighbors.cpu().numpy()[live], lref.neighbors[live]), st
        assert np.array_equal(eng.loader.t.cpu().numpy(), lref.t), st
        ins = np.unique(np.concatenate([s.src[sl], s.dst[sl]]))
        assert np.array_equal(eng.loader._assoc.cpu().numpy()[ins], np.arange(ins.size)), st
        _sync(ref, opt_ref, model, opt)
    ref.memory.train(False)
    eng.flush()
    torch.cuda.synchronize()
    assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5)
    assert torch.equal(model.memory.last_update.cpu(), ref.memory.last_update)
    # an eval batch of the same size (its update and insert use the partitioned plans too)
    from oracle.tgn_ref import eval_step
    a = nb * B   # the next batch (e_ids continue the stream)
    sl = slice(a, a + B)
    src, pos = torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl])
    negs = torch.from_numpy(rng.choice(s.dst_nodes, size=(B, 1)))
    po, no = eval_step(ref, lref, ev_t, ev_msg, src, pos, negs, ev_t[sl], ev_msg[sl])
    pg, ngm, rr = eng.eval_batch(a, B, negs)
    torch.cuda.synchronize()
    eng.check()
    assert torch.allclose(pg.cpu(), po, atol=2e-5) and torch.allclose(ngm.cpu(), no, atol=2e-5)
    assert torch.allclose(model.memory.memory.cpu(), ref.memory.memory, atol=1e-5)
    assert np.array_equal(eng.loader.e_id.cpu().numpy(), lref.e_id)


def test_tgn_pipelined_reprepares_after_loader_reset():
    """A pipelined step prepares the next batch from the ring (marking + scan); a host-side ring change through
    the loader between steps (here LastNeighborLoader.reset_state, neighbor_loader.py:106-109, called
    directly on the loader) bumps its version, so the next pipelined step prepares the batch again instead of
    using the stale scan.  Against a resident twin given the same reset: ring, outputs and memory."""
    engines = []
    for pipe in (True, False):
        s, ref, opt_ref, lref, model, opt, eng = _setup("last")
        model.cfg.dropout = 0.0
        eng.pipeline = pipe
        eng.bind_resident(0, 7 * 50, 50, dropout=False)
        eng.begin_epoch()
        if pipe:
            eng.capture_resident()
        engines.append((model, opt, eng))
    (m1, o1, e1), (m2, o2, e2) = engines
    for st in range(5):
        if st == 3:
            for e in (e1, e2):
                e.loader.reset_state()          # the ring is empty again; the prefetched scan saw it full
        e1.replay_resident()
        e2.resident_train_step()
        torch.cuda.synchronize()
        e1.check()
        e2.check()
        B = int(e2.ctl[2])
        assert torch.equal(e1.loader.e_id, e2.loader.e_id) and torch.equal(e1.loader.neighbors, e2.loader.neighbors), st
        assert torch.allclose(e1.out_pos[:B], e2.out_pos[:B], atol=1e-5), st
        assert torch.allclose(m1.memory.memory, m2.memory.memory, atol=1e-5), st
        with torch.no_grad():
            m1.flat.copy_(m2.flat)
            o1.exp_avg.copy_(o2.exp_avg)
            o1.exp_avg_sq.copy_(o2.exp_avg_sq)
            m1.memory.memory.copy_(m2.memory.memory)


def test_tgn_pp_wrong_parity_sets_error():
    """tgnx_tgn_train_step_pp with prefetched = 1 but the parity whose set holds the PREVIOUS batch: the
    step's first launch finds the set's batch tag stale, sets ctl[ERR] bit 16 and the step computes nothing
    (memory and parameters unchanged); check() raises."""
    s, ref, opt_ref, lref, model, opt, eng = _setup("last")
    eng.bind_resident(0, 7 * 50, 50, dropout=False)
    eng.begin_epoch()
    eng.resident_train_step()            # eager, parity 0; scans batch 1 into set 1
    torch.cuda.synchronize()
    eng.check()
    assert eng._parity == 1
    mem, flat = model.memory.memory.clone(), model.flat.clone()
    eng._pre(True, 0)                   # set 0 still holds batch 0
    torch.cuda.synchronize()
    assert int(eng.ctl[11]) & 16
    assert torch.equal(model.memory.memory, mem) and torch.equal(model.flat, flat)
    with pytest.raises(RuntimeError):
        eng.check()


def test_tgn_pp_refuses_foreign_plan_table():
    """The resident parity-set step refuses a plan table that tgnx_tgn_plan_table built for another split or
    batch (the slot index and stride would otherwise hand it another batch's plans or read past the
    table) and one the library did not build; nothing is launched (ctl untouched)."""
    import ctypes
    from tgnx import _lib
    s, ref, opt_ref, lref, model, opt, eng = _setup("last")
    eng.bind_resident(0, 7 * 50, 50, dropout=False)
    eng.begin_epoch()
    torch.cuda.synchronize()
    L = _lib.lib()
    ctl0 = eng.ctl.clone()
    # the engine's table is for [0, 350) batch 50: a step over [0, 300) or batch 40 must be refused
    for lo, hi, batch in ((0, 6 * 50, 50), (0, 7 * 50, 40), (50, 7 * 50, 50)):
        rc = L.tgnx_tgn_train_step_pp(eng._cfg_ref, eng._buf_ref, lo, hi, batch, 0, 0, 0, 0, eng._stream())
        assert rc != 0, (lo, hi, batch)
        assert "plan_table" in L.tgnx_last_error().decode()
    # a buffer of the right size the library never built a table in
    fake = torch.zeros_like(eng.plan_table)
    eng._res_buf.plan_table = fake.data_ptr()
    rc = L.tgnx_tgn_train_step_pp(eng._cfg_ref, eng._buf_ref, 0, 7 * 50, 50, 0, 0, 0, 0, eng._stream())
    assert rc != 0 and "not built" in L.tgnx_last_error().decode()
    eng._res_buf.plan_table = eng.plan_table.data_ptr()
    torch.cuda.synchronize()
    assert torch.equal(eng.ctl, ctl0)
    eng.resident_train_step()            # the matching table still works
    torch.cuda.synchronize()
    eng.check()


def test_tgn_engine_matches_reference_model_wiring():
    """The HIP step against the reference's own model wiring (tests/golden/tgn_model_wiring.npz:
    pyg_model_utils.getModel as written, GraphAttentionEmbedding emb_module.py:11-29, LinkPredictor, the
    reference LastNeighborLoader; make_goldens.py capture_tgn_model), 4 batches with Adam, nothing
    resynchronised: outputs 2e-5, loss, every gradient 2e-3 relative (lin_key.bias: negligible on both sides),
    memory 1e-5, last_update exact."""
    import os
    from tgnx.sampler import LastNeighborLoader
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "tgn_model_wiring.npz"))
    N, d, D, B, nb = z["meta"].tolist()
    dev = torch.device("cuda")
    model = TGNModel(N, nb * B, d, D, dev, ring=10, max_batch=B, max_neg=1, aggr="last", dropout=0.0)
    sd = {k[2:].replace("__", ".", 1).replace("__", "."): torch.from_numpy(z[k]) for k in z.files if k.startswith("p_")}
    model.load_reference_state(sd)
    opt = TgnAdam(model, float(z["lr"][0]))
    eng = TgnEngine(model, LastNeighborLoader(N, 10, device=dev),
                    dict(src=z["src"].reshape(-1), dst=z["dst"].reshape(-1), t=z["t"].reshape(-1).astype(np.float32),
                         msg=z["msg"]), opt, dst_nodes=np.unique(z["dst"]))
    eng.reset_state()
    for b in range(nb):
        pg, ng = eng.train_batch(b * B, B, neg=torch.from_numpy(z["neg"][b]), dropout=False)
        torch.cuda.synchronize()
        eng.check()
        assert np.allclose(pg.cpu().numpy(), z[f"b{b}_pos"], atol=2e-5), b
        assert np.allclose(ng.cpu().numpy(), z[f"b{b}_neg"], atol=2e-5), b
        assert abs(float(model.grad_flat[-1]) - float(z[f"b{b}_loss"][0])) < 1e-5, b
        g = model.grads_by_name()
        for name in model.param_order:
            want = torch.from_numpy(z[f"b{b}_g_" + name.replace(".", "__")])
            if name in SHIFT_INVARIANT:
                scale = float(torch.from_numpy(z[f"b{b}_g_" + SHIFT_INVARIANT[name].replace(".", "__")]).norm())
                assert float(g[name].norm()) <= 1e-4 * scale + 1e-9, (b, name)
                continue
            if float(want.norm()) == 0.0:
                assert float(g[name].norm()) < 1e-7, (b, name)
                continue
            r = _rel(g[name], want)
            assert r < 2e-3, (b, name, r)
        assert np.allclose(model.memory.memory.cpu().numpy(), z[f"b{b}_memory"], atol=1e-5), b
        assert np.array_equal(model.memory.last_update.cpu().numpy(), z[f"b{b}_last_update"]), b


def test_tgn_no_grad_store_same_step():
    """TGNX_TGN_NO_GRAD_STORE (TgnEngine.keep_grads = False, what bench.py and the drop-in train() run): the
    replayed parity-set steps with Adam fused leave the gradient buffer untouched (the loss slot aside) and
    produce the same parameters, moments, memory, outputs and loss as the same steps storing it — within the
    run-to-run spread of the float atomics' order (dZc / hub dP sums), as the other step-form comparisons."""
    from tgnx.sampler import LastNeighborLoader
    from tgnx.tgn import TgnAdam, TgnEngine, TGNModel
    s, ref, opt_ref, lref, model, opt, eng = _setup("last")
    dev = torch.device("cuda")
    sd = ref.state_dict()
    engs = []
    for keep in (True, False):
        m = TGNModel(300, s.num_events, 16, 32, dev, ring=10, max_batch=50, max_neg=1, aggr="last", dropout=0.1)
        m.load_reference_state(sd)
        e = TgnEngine(m, LastNeighborLoader(300, 10, device=dev), dict(src=s.src, dst=s.dst,
                      t=s.t.astype(np.float32), msg=s.msg), TgnAdam(m, 1e-3), dst_nodes=s.dst_nodes, seed=5)
        e.keep_grads = keep
        e.bind_resident(0, 8 * 50, 50, dropout=True)
        e.begin_epoch()
        e.capture_resident()
        m.grad_flat.fill_(7.0)
        engs.append(e)
    for st in range(8):
        for e in engs:
            e.replay_resident()
        torch.cuda.synchronize()
        a, b = engs
        a.check()
        b.check()
        for name in a.model.param_order:
            if name in SHIFT_INVARIANT:
                continue
            o, n, _ = a.model._views[name]
            assert _rel(b.model.flat[o:o + n], a.model.flat[o:o + n]) < 1e-5, (st, name)
            assert _rel(b.adam_m[o:o + n], a.adam_m[o:o + n]) < 1e-4, (st, name)
        assert torch.allclose(a.model.memory.memory, b.model.memory.memory, atol=1e-5), st
        assert torch.equal(a.model.memory.last_update, b.model.memory.last_update), st
        assert torch.allclose(a.out_pos, b.out_pos, atol=1e-5) and torch.allclose(a.out_neg, b.out_neg, atol=1e-5), st
        assert abs(a.loss_sum() - b.loss_sum()) <= 1e-5 * max(1.0, abs(a.loss_sum())), st
        G = b.model.grad_flat
        assert torch.all(G[:-1] == 7.0), st                    # never stored
        assert not torch.all(a.model.grad_flat[:-1] == 7.0), st
        with pytest.raises(RuntimeError, match="keep_grads"):  # stale gradients are not handed out
            b.model.grads_by_name()
        assert a.model.grads_by_name()
        with torch.no_grad():   # re-synchronise (the wiki time scale turns ulp differences chaotic)
            b.model.flat.copy_(a.model.flat)
            b.adam_m.copy_(a.adam_m)
            b.adam_v.copy_(a.adam_v)
            b.model.memory.memory.copy_(a.model.memory.memory)
