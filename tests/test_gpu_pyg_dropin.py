"""GPU test of the PyG TGN drop-in (tgb-tgn-dgl_amd/pyg_model_utils.py + pyg_epoch_utils.py, the seam of
pyg-mem-tgn.py:23-25 "#change based on dgl/pyg"): one train epoch and one validation pass through the
reference's train / test signatures on a small wiki-shaped stream.

Checks: the first train batch against the oracle's canonical step (oracle/tgn_ref.train_step, same
device-drawn negatives, dropout off); train() returns Σ loss·B of its batches; the first test() after
training flushes the memory (TGNMemory.train(False): stores empty, memory_module.py:209-215); test()
returns the mean over batches of the per-event TGB reciprocal ranks."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pyg_dropin_epoch(monkeypatch):
    monkeypatch.setenv("TGNX_SYNTH_EVENTS", "3000")
    monkeypatch.setenv("TGNX_EVAL_NEGS", "30")
    import pyg_epoch_utils as pe
    import pyg_model_utils as pm
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, train_step
    from tgnx.data import getDataWithDependecyBlock
    from tgnx.neg import NegLinkSamplerDest
    from tgnx.sampler import LastNeighborLoader
    data, tr, va, te, ns, ev, metric = getDataWithDependecyBlock("tgbl-wiki", {"batch_size": 200})
    d, D, N = data.msg.shape[1], 100, data.num_nodes
    torch.manual_seed(0)
    ref = RefTGN(N, d, hidden=D, aggr="last", dropout=0.0)
    model = pm.getModel(d, D, N, "cuda", ring=10, max_batch=200, dropout=0.0)
    model["model"].load_reference_state(ref.state_dict())
    opt = pm.getOptimizer(model, 1e-4)
    nl = LastNeighborLoader(N, 10, device="cuda")
    nds = NegLinkSamplerDest(torch.unique(data.dst), device="cuda")
    crit = torch.nn.BCEWithLogitsLoss()
    total = pe.train(model, data.msg, tr, nl, nds, None, "cuda", opt, crit)
    eng = model["model"]._tgnx_engine
    assert np.isfinite(total) and total > 0
    assert abs(total - eng.loss_sum()) < 1e-6 * max(1.0, abs(total))

    # the first batch again on a fresh engine + the oracle, with the negatives the device drew
    B = 200
    neg = eng.neg_train[tr.lo:tr.lo + B].cpu()
    m2 = pm.getModel(d, D, N, "cuda", ring=10, max_batch=200, dropout=0.0)
    m2["model"].load_reference_state(ref.state_dict())
    from tgnx.tgn import TgnEngine
    e2 = TgnEngine(m2["model"], LastNeighborLoader(N, 10, device="cuda"),
                   dict(src=data.src, dst=data.dst, t=data.t.float(), msg=data.msg.float()), pm.getOptimizer(m2, 1e-4),
                   dst_nodes=torch.unique(data.dst))
    e2.reset_state()
    pg, ng = e2.train_batch(tr.lo, B, neg=neg)
    ev_t, ev_msg = data.t.float(), data.msg.float()
    sl = slice(tr.lo, tr.lo + B)
    _, po, no = train_step(ref, torch.optim.Adam(ref.parameters(), lr=1e-4), RefLastNeighborLoader(N, 10), ev_t, ev_msg,
                           data.src[sl], data.dst[sl], neg, ev_t[sl], ev_msg[sl])
    torch.cuda.synchronize()
    assert torch.allclose(pg.cpu(), po, atol=2e-5) and torch.allclose(ng.cpu(), no, atol=2e-5)

    # validation: flush on the first test() call, then per-event TGB MRR
    mrr = pe.test(model, data.msg, va, nl, ns, None, "cuda", opt, crit, ev, metric, "val")
    assert 0.0 < mrr <= 1.0
    assert int(model["model"].store[:4 * N].view(N, 4)[:, [1, 3]].sum()) > 0   # eval batches re-filled the stores
    # a second test() call does not flush again and scores the next split with the same state rules
    mrr2 = pe.test(model, data.msg, te, nl, ns, None, "cuda", opt, crit, ev, metric, "test")
    assert 0.0 < mrr2 <= 1.0
