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
