"""CPU tests of the TGB on-disk loader (tgnx.tgb_io; SURVEY §8f.2, utils.py:25-67 via py-tgb).  py-tgb and
TGB files are absent, so these pin tgnx's restatement of py-tgb's conventions (PARITY UNPINNED against
py-tgb itself): JODIE-layout wiki CSV (item ids shifted past the users), generic edge lists relabelled
in order of appearance, quantile splits (generate_splits), the npz cache, pickled negatives read only
with allow_pickle, and the reference surface getDataWithDependecyBlock picking the on-disk stream."""
import os
import pickle

import numpy as np
import pytest

from tgnx import tgb_io


def _wiki_csv(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "tgbl-wiki_edgelist_v2.csv"), "w") as f:
        f.write("user_id,item_id,timestamp,state_label,comma_separated_list_of_features\n")
        for u, i, t, fe in rows:
            f.write(",".join([str(u), str(i), str(t), "0"] + [repr(x) for x in fe]) + "\n")


def test_split_bounds_match_quantile_masks():
    rng = np.random.default_rng(0)
    t = np.sort(rng.integers(0, 50, 1000)).astype(np.float64)   # many ties at the quantiles
    tr, va = tgb_io.split_bounds(t)
    vt, tt = np.quantile(t, [0.70, 0.85])
    assert np.array_equal(np.arange(1000) < tr, t <= vt)
    assert np.array_equal((np.arange(1000) >= tr) & (np.arange(1000) < va), (t > vt) & (t <= tt))
    assert np.array_equal(np.arange(1000) >= va, t > tt)
    with pytest.raises(ValueError):
        tgb_io.split_bounds(np.array([3.0, 1.0]))


def test_wiki_csv_layout_and_cache(tmp_path):
    rng = np.random.default_rng(1)
    rows = [(int(rng.integers(0, 5)), int(rng.integers(0, 3)), 10 * k, rng.random(4).round(6).tolist()) for k in range(40)]
    d = tgb_io.dataset_dir("tgbl-wiki", str(tmp_path))
    _wiki_csv(d, rows)
    src, dst, t, msg, tr, va, negs = tgb_io.load_tgb("tgbl-wiki", str(tmp_path))
    umax = max(r[0] for r in rows)
    assert np.array_equal(src, [r[0] for r in rows])
    assert np.array_equal(dst, [r[1] + umax + 1 for r in rows])
    assert np.array_equal(t, [r[2] for r in rows])
    assert np.allclose(msg, np.asarray([r[3] for r in rows], np.float32))
    assert (tr, va) == tgb_io.split_bounds(t) and negs == {}
    assert os.path.exists(os.path.join(d, "tgnx_tgbl-wiki.npz"))
    again = tgb_io.load_tgb("tgbl-wiki", str(tmp_path))            # from the cache
    for a, b in zip(again[:4], (src, dst, t, msg)):
        assert np.array_equal(a, b)
    assert again[4:6] == (tr, va)


def test_edgelist_relabel_and_pickled_negatives(tmp_path):
    d = tgb_io.dataset_dir("tgbl-review", str(tmp_path))
    os.makedirs(d)
    keys = ["a", "b", "c", "x", "y", "d"]
    ev = [(5 + k // 2, keys[(3 * k) % 6], keys[(5 * k + 1) % 6], 0.5 * k) for k in range(24)]
    ev = [e for e in ev if e[1] != e[2]]
    with open(os.path.join(d, "tgbl-review_edgelist_v2.csv"), "w") as f:
        f.write("ts,src,dst,w\n")
        for t, s, dd, w in ev:
            f.write(f"{t},{s},{dd},{w}\n")
    ids = {}
    for _, s, dd, _ in ev:
        ids.setdefault(s, len(ids))
        ids.setdefault(dd, len(ids))
    src, dst, t, msg = tgb_io.read_edgelist_csv(os.path.join(d, "tgbl-review_edgelist_v2.csv"))
    assert np.array_equal(src, [ids[e[1]] for e in ev]) and np.array_equal(dst, [ids[e[2]] for e in ev])
    assert np.array_equal(msg[:, 0], [e[3] for e in ev])
    tr, va = tgb_io.split_bounds(t)
    table = {(int(src[e]), int(dst[e]), int(t[e])): [100 + e, 200 + e, 300 + e][: 2 + (e % 2)] for e in range(len(ev))}
    for split in ("val", "test"):
        with open(os.path.join(d, f"tgbl-review_{split}_ns.pkl"), "wb") as f:   # our own file
            pickle.dump(table, f)
    with pytest.raises(RuntimeError):
        tgb_io.load_tgb("tgbl-review", str(tmp_path))
    *_, negs = tgb_io.load_tgb("tgbl-review", str(tmp_path), allow_pickle=True)
    for split, lo, hi in (("val", tr, va), ("test", va, len(ev))):
        k = min(len(table[(int(src[e]), int(dst[e]), int(t[e]))]) for e in range(lo, hi))
        want = np.asarray([table[(int(src[e]), int(dst[e]), int(t[e]))][:k] for e in range(lo, hi)])
        assert np.array_equal(negs[f"{split}_neg"], want)
    # the cache (plain arrays) now serves without the pickles
    for split in ("val", "test"):
        os.remove(os.path.join(d, f"tgbl-review_{split}_ns.pkl"))
    *_, negs2 = tgb_io.load_tgb("tgbl-review", str(tmp_path))
    assert np.array_equal(negs2["val_neg"], negs["val_neg"])


def test_reference_surface_reads_the_disk_stream(tmp_path, monkeypatch):
    from tgnx.data import getDataWithDependecyBlock
    rng = np.random.default_rng(2)
    rows = [(int(rng.integers(0, 6)), int(rng.integers(0, 4)), 5 * k, rng.random(3).tolist()) for k in range(60)]
    _wiki_csv(tgb_io.dataset_dir("tgbl-wiki", str(tmp_path)), rows)
    monkeypatch.setenv("TGNX_TGB_ROOT", str(tmp_path))
    monkeypatch.setenv("TGNX_EVAL_NEGS", "7")
    data, tr_dl, va_dl, te_dl, ns, ev, metric = getDataWithDependecyBlock("tgbl-wiki", {"batch_size": 10})
    assert data.num_events == 60 and metric == "mrr"
    assert np.array_equal(data.src.numpy(), [r[0] for r in rows])
    tr, va = tgb_io.split_bounds(np.asarray([r[2] for r in rows], np.float64))
    assert (tr_dl.lo, tr_dl.hi, va_dl.lo, va_dl.hi, te_dl.hi) == (0, tr, tr, va, 60)
    neg = ns.query_batch(data.src[tr:tr + 3], data.dst[tr:tr + 3], None, split_mode="val")
    assert len(neg) == 3 and all(len(r) == 7 for r in neg)
    assert all(int(data.dst[tr + i]) not in r for i, r in enumerate(neg))
