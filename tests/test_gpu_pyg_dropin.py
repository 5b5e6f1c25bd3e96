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


def _write_cfg(path, mail_combine, batch=None):
    import yaml
    src = open(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "tgb-tgn-dgl_amd", "config",
                                           "TGN.yml")).read()
    conf = yaml.safe_load(src)
    conf["memory"][0]["mail_combine"] = mail_combine
    conf["train"][0]["epoch"] = 1
    if batch is not None:
        conf["train"][0]["batch_size"] = batch
    with open(path, "w") as f:
        yaml.safe_dump(conf, f)
    return str(path)


def test_reference_script_with_one_line_swap(tmp_path, monkeypatch):
    """The reference's entry script (/root/reference/pyg-mem-tgn.py:16-63) with only its model import swapped
    (:24 -> :25), run call for call through the shims: parse_config, getDataWithDependecyBlock,
    NegLinkSamplerDest(unique destinations) without a device, LastNeighborLoader, getModel(d, dim_out, N,
    device, gnn_param=gnn_param), getOptimizer, and epoch_utils.train / test (NOT pyg_epoch_utils: :19
    keeps the DGL loop's import, which dispatches on the model dict).  The config says mail_combine 'mean';
    the model must be the MeanAggregator TGN: a fresh getModel from the same gnn_param, on two batches
    with injected negatives and dropout off, matches oracle RefTGN(aggr='mean') and not aggr='last'.  The batch
    size is TGN.yml's own (config/TGN.yml:27, batch_size 2000): two full batches and a partial one per epoch."""
    monkeypatch.setenv("TGNX_SYNTH_EVENTS", "8000")
    monkeypatch.setenv("TGNX_EVAL_NEGS", "20")
    from dependencyGraph import dependecyAwareBatch as dab  # noqa: F401  (imported by the script, :17)
    from epoch_utils import test, train
    from neg_sampler import NegLinkSamplerDest
    from neighbor_loader import LastNeighborLoader
    from pyg_model_utils import getModel, getOptimizer
    from utils import getDataWithDependecyBlock, parse_config
    cfg = _write_cfg(tmp_path / "TGN_mean.yml", "mean")
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    sample_param, memory_param, gnn_param, train_param = parse_config(cfg)
    data, train_dataloader, val_dataloader, test_dataloader, neg_sampler, evaluator, metric = \
        getDataWithDependecyBlock("tgbl-wiki", train_param)
    unique_destination_nodes = torch.unique(data.dst)
    neg_dest_sampler = NegLinkSamplerDest(unique_destination_nodes)
    assoc = torch.empty(data.num_nodes, dtype=torch.long, device=device)
    neighbor_loader = LastNeighborLoader(data.num_nodes, size=sample_param["neighbor"][0], device=device)
    model = getModel(data.msg.shape[1], gnn_param["dim_out"], data.num_nodes, device, gnn_param=gnn_param)
    optimizer = getOptimizer(model, train_param["lr"])
    criterion = torch.nn.BCEWithLogitsLoss()
    m = model["model"]
    assert set(model) >= {"memory", "gnn", "link_pred"}
    assert m.cfg.aggr == 1 and m.layers == 1 and m.updater == "gru" and m.cfg.max_batch == 2000 and m.cfg.ring == 10
    assert train_param["batch_size"] == 2000
    for e in range(train_param["epoch"]):
        loss = train(model, data.msg, train_dataloader, neighbor_loader, neg_dest_sampler, assoc, device, optimizer,
                     criterion)
        assert np.isfinite(loss) and loss > 0
        mrr = test(model, data.msg, val_dataloader, neighbor_loader, neg_sampler, assoc, device, optimizer, criterion,
                   evaluator, metric, "val")
        assert 0.0 < mrr <= 1.0
    assert m._tgnx_engine.loss_sum() > 0

    # the selection is the MeanAggregator: oracle parity with aggr='mean' (and a mismatch with 'last')
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, train_step
    from tgnx.tgn import TgnEngine
    N, d, D, B = data.num_nodes, data.msg.shape[1], gnn_param["dim_out"], train_param["batch_size"]
    torch.manual_seed(0)
    refs = {a: RefTGN(N, d, hidden=D, aggr=a, dropout=0.0) for a in ("mean", "last")}
    refs["last"].load_state_dict(refs["mean"].state_dict())
    m2 = getModel(d, D, N, device, gnn_param=gnn_param, dropout=0.0)
    m2["model"].load_reference_state(refs["mean"].state_dict())
    e2 = TgnEngine(m2["model"], LastNeighborLoader(N, 10, device=device),
                   dict(src=data.src, dst=data.dst, t=data.t.float(), msg=data.msg.float()), getOptimizer(m2, 1e-4),
                   dst_nodes=unique_destination_nodes)
    e2.reset_state()
    opts = {a: torch.optim.Adam(r.parameters(), lr=1e-4) for a, r in refs.items()}
    lrefs = {a: RefLastNeighborLoader(N, 10) for a in refs}
    ev_t, ev_msg = data.t.float(), data.msg.float()
    rng = np.random.default_rng(3)
    diff_last = 0.0
    for st in range(2):
        sl = slice(st * B, (st + 1) * B)
        neg = torch.from_numpy(rng.choice(unique_destination_nodes.numpy(), size=B))
        pg, ng = e2.train_batch(st * B, B, neg=neg)
        torch.cuda.synchronize()
        outs = {a: train_step(refs[a], opts[a], lrefs[a], ev_t, ev_msg, data.src[sl], data.dst[sl], neg, ev_t[sl],
                              ev_msg[sl]) for a in refs}
        _, po, no = outs["mean"]
        assert torch.allclose(pg.cpu(), po, atol=2e-5) and torch.allclose(ng.cpu(), no, atol=2e-5), st
        diff_last = max(diff_last, float((pg.cpu() - outs["last"][1]).abs().max()))
    assert diff_last > 1e-3   # the two aggregations differ on this stream: the match above selects 'mean'


def test_dropin_train_twice_with_test_between_matches_oracle(tmp_path):
    """The drop-in train() as the reference script calls it, twice, with test() between: the graphs
    captured in epoch 1 are replayed in epoch 2 after begin_epoch / flush / eval ran on the same buffers.  Every
    step of both epochs is checked — without resynchronisation — through the per-event output log (out_ev)
    against oracle/tgn_ref.train_step fed the negatives the device drew (eng.neg_train after each epoch), on a
    wiki-shaped stream whose timestamps span 2,000 s (not chaotic: DESIGN §7), dropout off.  Tolerances:
    per-event outputs 1e-4 abs, train() loss sums 1e-4 relative, val MRR 5e-3 (test_gpu_tgn_epochs.py's)."""
    import pyg_epoch_utils as pe
    import pyg_model_utils as pm
    from epoch_parity import scaled_stream
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, eval_step, mrr_per_event, train_step
    from tgnx.data import getDataWithDependecyBlock
    from tgnx.neg import NegLinkSamplerDest
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import eval_negatives
    s = scaled_stream(4, N=1000, E=3000, d=16, t_max=2000)
    path = str(tmp_path / "short.npz")
    np.savez(path, src=s.src, dst=s.dst, t=s.t, msg=s.msg, val_neg=eval_negatives(s, "val", 30),
             test_neg=eval_negatives(s, "test", 30))
    B = 200
    data, tr, va, te, ns, ev, metric = getDataWithDependecyBlock(path, {"batch_size": B})
    d, D, N = data.msg.shape[1], 100, data.num_nodes
    torch.manual_seed(0)
    ref = RefTGN(N, d, hidden=D, aggr="last", dropout=0.0)
    model = pm.getModel(d, D, N, "cuda", ring=10, max_batch=B, dropout=0.0)
    model["model"].load_reference_state(ref.state_dict())
    opt = pm.getOptimizer(model, 1e-4)
    nl = LastNeighborLoader(N, 10, device="cuda")
    nds = NegLinkSamplerDest(torch.unique(data.dst), device="cuda")
    crit = torch.nn.BCEWithLogitsLoss()
    runs = []
    for ep in range(2):
        loss = pe.train(model, data.msg, tr, nl, nds, None, "cuda", opt, crit)
        eng = model["model"]._tgnx_engine
        runs.append(dict(loss=loss, neg=eng.neg_train[tr.lo:tr.hi].cpu().clone(),
                         out=eng.out_ev[tr.lo:tr.hi].cpu().clone()))
        runs[-1]["mrr"] = pe.test(model, data.msg, va, nl, ns, None, "cuda", opt, crit, ev, metric, "val")
    assert model["model"]._tgnx_engine._graphs is not None
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-4)
    ev_t, ev_msg = data.t.float(), data.msg.float()
    vneg = va.negatives
    for ep, run in enumerate(runs):
        ref.memory.reset_state()
        ref.memory.train(True)
        lref = RefLastNeighborLoader(N, 10)
        tot = 0.0
        for a in range(tr.lo, tr.hi, B):
            b = min(a + B, tr.hi)
            sl = slice(a, b)
            loss, po, no = train_step(ref, opt_ref, lref, ev_t, ev_msg, data.src[sl], data.dst[sl],
                                      run["neg"][a - tr.lo:b - tr.lo], ev_t[sl], ev_msg[sl])
            tot += loss * (b - a)
            got = run["out"][a - tr.lo:b - tr.lo]
            assert torch.allclose(got[:, 0], po, atol=1e-4), (ep, a, float((got[:, 0] - po).abs().max()))
            assert torch.allclose(got[:, 1], no, atol=1e-4), (ep, a, float((got[:, 1] - no).abs().max()))
        assert abs(run["loss"] - tot) <= 1e-4 * abs(tot), (ep, run["loss"], tot)
        ref.memory.train(False)
        per = []
        for a in range(va.lo, va.hi, B):
            b = min(a + B, va.hi)
            sl = slice(a, b)
            po, no = eval_step(ref, lref, ev_t, ev_msg, data.src[sl], data.dst[sl], vneg[a - va.lo:b - va.lo],
                               ev_t[sl], ev_msg[sl])
            per.append(float(np.mean(mrr_per_event(po, no))))
        assert abs(run["mrr"] - float(np.mean(per))) < 5e-3, (ep, run["mrr"], float(np.mean(per)))
