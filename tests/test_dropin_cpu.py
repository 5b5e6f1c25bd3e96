"""CPU tests of the drop-in surface (no GPU): config schema, data/batching semantics,
native dependency blocks vs the oracle, evaluator rank rule."""
import os

import numpy as np
import pytest
import torch

from conftest import PKG


def test_parse_config_schema():
    from utils import parse_config
    s, m, g, t = parse_config(os.path.join(PKG, "config", "TGN.yml"))
    assert s["neighbor"][0] == 10 and g["dim_out"] == 100 and g["att_head"] == 8 and g["layer"] == 1
    assert t["batch_size"] == 2000 and t["lr"] == 1e-4 and t["epoch"] == 3000
    assert m["mail_combine"] == "last" and m["memory_update"] == "gru"


def test_native_blocks_match_oracle_on_wiki_shaped_stream():
    from oracle import blocks_ref
    from tgnx.data import block_ids
    from tgnx.synth import make_stream
    s = make_stream("tgbl-wiki", seed=3, num_events=20_000)
    for B in (200, 600, 2000):
        np.testing.assert_array_equal(block_ids(s.src, s.dst, B), blocks_ref.block_ids(s.src, s.dst, B))


def test_get_block_and_dab_api(golden):
    from dependencyGraph import dependecyAwareBatch, get_block
    z = golden("blocks.npz")
    assert get_block([0.0] * 6, [1, 1, 2, 3, 3, 5], [2, 4, 4, 1, 5, 1]) == z["small"].tolist()
    B = int(z["batch"][0])
    loader = [{"src": torch.from_numpy(z["src"][i:i + B]), "dst": torch.from_numpy(z["dst"][i:i + B]),
               "t": torch.from_numpy(z["t"][i:i + B])} for i in range(0, z["src"].shape[0], B)]
    np.testing.assert_array_equal(np.array(dependecyAwareBatch(loader, flat=True)), z["blocks"])


def test_temporal_dataset_matches_golden_collate(golden):
    from torch.utils.data import DataLoader

    from temporal_dataset import TemporalGraphDataset
    z = golden("dataset.npz")
    ds = TemporalGraphDataset(torch.from_numpy(z["in_src"]), torch.from_numpy(z["in_dst"]),
                              torch.from_numpy(z["in_t"]), torch.from_numpy(z["in_msg"]), batch=list(z["in_b"]))
    rec = {k: [] for k in ("src", "dst", "t", "msg", "b", "idx")}
    for b in DataLoader(ds, batch_size=10, shuffle=False):
        for k in rec:
            rec[k].append(b[k].numpy())
    for k in rec:
        got = np.concatenate(rec[k])
        np.testing.assert_array_equal(got, z[k])
        assert got.dtype == z[k].dtype, k


def test_get_data_splits_blocks_and_negatives(monkeypatch):
    monkeypatch.setenv("TGNX_SYNTH_EVENTS", "3000")
    monkeypatch.setenv("TGNX_EVAL_NEGS", "20")
    from oracle import blocks_ref
    from utils import getDataWithDependecyBlock
    data, tr, va, te, ns, ev, metric = getDataWithDependecyBlock("tgbl-wiki", {"batch_size": 200})
    assert metric == "mrr" and data.num_events == 3000
    E = data.num_events
    assert (tr.lo, tr.hi, va.lo, va.hi, te.lo, te.hi) == (0, 2100, 2100, 2550, 2550, 3000)
    np.testing.assert_array_equal(tr.blocks.numpy(), blocks_ref.block_ids(data.src[:2100].numpy(),
                                                                           data.dst[:2100].numpy(), 200))
    # utils.py:55-61 quirk: val batches carry the test split's block ids and vice versa
    np.testing.assert_array_equal(va.blocks.numpy(), blocks_ref.block_ids(data.src[2550:].numpy(),
                                                                          data.dst[2550:].numpy(), 200))
    b0 = next(iter(tr))
    assert b0["t"].dtype == torch.float32 and b0["src"].dtype == torch.long and b0["msg"].shape == (200, 172)
    assert sum(b["src"].shape[0] for b in tr) == 2100 and len(tr) == 11
    rows = ns.query_batch(b0["src"], b0["dst"], b0["t"], split_mode="val")
    assert len(rows) == 200 and all(len(r) == 20 for r in rows)
    vneg = va.negatives.numpy()
    assert (vneg != data.dst[2100:2550].numpy()[:, None]).all()   # true negatives
    assert E == 3000


def test_evaluator_rank_rule():
    from oracle.mrr_ref import mrr_batch
    from utils import Evaluator
    rng = np.random.default_rng(0)
    pos = rng.standard_normal(50).astype(np.float32)
    neg = rng.standard_normal((50, 30)).astype(np.float32)
    neg[3, :5] = pos[3]          # ties count half
    got = Evaluator("x").eval({"y_pred_pos": pos, "y_pred_neg": neg, "eval_metric": ["mrr"]})["mrr"]
    assert abs(got - mrr_batch(pos, neg)) < 1e-12


def test_product_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from tgnx.sampler import LastNeighborLoader
    with pytest.raises(RuntimeError, match="HIP device"):
        LastNeighborLoader(10, 3, device="cpu")


def test_config_sections_select_the_tgn_model(tmp_path):
    """pyg-mem-tgn.py:36,49 passes only gnn_param to getModel; tgnx's parse_config records the file so that
    pyg_model_utils.getModel honours the memory section (config/TGN.yml:10-18: mail_combine, memory_update),
    sampling.neighbor[0] and train.batch_size.  Host logic only (no model is built)."""
    import yaml

    from tgnx.data import config_of, parse_config
    from tgnx.tgn import model_options
    src = os.path.join(PKG, "config", "TGN.yml")
    s, mem, g, tr = parse_config(src)
    assert config_of(g)[1] is mem
    assert model_options(g) == {"layers": 1, "aggr": "last", "updater": "gru", "ring": 10, "max_batch": 2000}
    conf = yaml.safe_load(open(src))
    conf["memory"][0].update(mail_combine="mean", memory_update="rnn")
    conf["gnn"][0]["layer"] = 2
    conf["sampling"][0]["neighbor"] = [20]
    p = tmp_path / "c.yml"
    yaml.safe_dump(conf, open(p, "w"))
    s2, mem2, g2, tr2 = parse_config(str(p))
    assert model_options(g2) == {"layers": 2, "aggr": "mean", "updater": "rnn", "ring": 20, "max_batch": 2000}
    # a gnn dict that did not come from parse_config: only its own keys
    assert model_options(dict(g2)) == {"layers": 2}
    assert model_options(dict(g2), memory_param=dict(mem2)) == {"layers": 2, "aggr": "mean", "updater": "rnn"}
    with pytest.raises(ValueError):
        model_options(g2, memory_param=dict(mem2, mail_combine="max"))
    with pytest.raises(NotImplementedError):
        model_options(g2, memory_param=dict(mem2, type="none"))


def test_batched_ap_auc_matches_sklearn():
    """tgnx.tgn_epoch.ap_auc_rows / epoch_ap_auc (the drop-in train()'s AP / AUC display, computed for every
    batch of the epoch at once from the per-event output log) against sklearn's average_precision_score /
    roc_auc_score per batch (pyg_epoch_utils.py:139-145), with tied scores, a partial last batch and the
    reference's extra sigmoid."""
    import numpy as np
    import torch
    from sklearn.metrics import average_precision_score, roc_auc_score

    from tgnx.tgn_epoch import ap_auc_rows, epoch_ap_auc
    rng = np.random.default_rng(0)
    for R, P, N, levels in ((7, 50, 50, 12), (3, 200, 200, 1000), (5, 9, 13, 3)):
        pos = torch.from_numpy(rng.integers(0, levels, (R, P)).astype(np.float32) / levels)
        neg = torch.from_numpy(rng.integers(0, levels, (R, N)).astype(np.float32) / levels)
        ap, auc = ap_auc_rows(pos, neg, chunk_elems=1000)
        for r in range(R):
            y = np.r_[np.ones(P), np.zeros(N)]
            sc = np.r_[pos[r].numpy(), neg[r].numpy()]
            assert abs(float(ap[r]) - average_precision_score(y, sc)) < 1e-12, (R, r)
            assert abs(float(auc[r]) - roc_auc_score(y, sc)) < 1e-12, (R, r)
    out_ev = torch.from_numpy(rng.random((1030, 2), dtype=np.float32))
    lo, hi, B = 10, 1030, 200
    aps, aucs = [], []
    for a in range(lo, hi, B):
        b = min(a + B, hi)
        y_pred = torch.cat([out_ev[a:b, 0], out_ev[a:b, 1]]).sigmoid()
        y_true = torch.cat([torch.ones(b - a), torch.zeros(b - a)])
        aps.append(average_precision_score(y_true, y_pred))
        aucs.append(roc_auc_score(y_true, y_pred))
    ap, auc = epoch_ap_auc(out_ev, lo, hi, B)
    assert abs(ap - float(np.mean(aps))) < 1e-12 and abs(auc - float(np.mean(aucs))) < 1e-12
