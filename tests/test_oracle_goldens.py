"""Pin the oracle against the golden vectors captured from the reference's own modules."""
import numpy as np
import pytest
import torch

from oracle import blocks_ref, negs_ref
from oracle.sampler_ref import RefLastNeighborLoader
from oracle.tgnn_ref import RefEdgePredictor, RefTimeEncode


def replay_sampler(z, loader_cls):
    N, K, nb, B, _ = z["meta"].tolist()
    ld = loader_cls(N, K)
    for bi in range(nb):
        q0 = z["q_off"][bi]
        q1 = z["q_off"][bi + 1] if bi + 1 < nb else z["q"].shape[0]
        n0 = z["nid_off"][bi]
        n1 = z["nid_off"][bi + 1] if bi + 1 < nb else z["nid"].shape[0]
        e0 = z["e_off"][bi]
        e1 = z["e_off"][bi + 1] if bi + 1 < nb else z["eid"].shape[0]
        nid, ei, eid, et = ld(z["q"][q0:q1])
        yield "call", bi, (nid, ei, eid, et, ld), (z["nid"][n0:n1], z["ei"][e0:e1].T, z["eid"][e0:e1],
                                                  z["et"][e0:e1], z["assoc_nid"][n0:n1])
        i0 = z["ins_off"][bi]
        ld.insert(z["ins_src"][i0:i0 + B], z["ins_dst"][i0:i0 + B], z["ins_t"][i0:i0 + B])
        yield "insert", bi, ld, (z["state_eid"][bi], z["state_t"][bi], z["state_nbr"][bi])


def _as_np(x):
    return x.cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def check_sampler_replay(z, loader_cls):
    n_calls = 0
    for kind, bi, got, want in replay_sampler(z, loader_cls):
        if kind == "call":
            nid, ei, eid, et, ld = got
            np.testing.assert_array_equal(_as_np(nid), want[0])
            np.testing.assert_array_equal(_as_np(ei), want[1])
            np.testing.assert_array_equal(_as_np(eid), want[2])
            np.testing.assert_array_equal(_as_np(et), want[3])
            np.testing.assert_array_equal(_as_np(ld._assoc)[want[0]], want[4])
            n_calls += 1
        else:
            eid = _as_np(got.e_id)
            np.testing.assert_array_equal(eid, want[0])
            np.testing.assert_array_equal(_as_np(got.t), want[1])
            nbr = _as_np(got.neighbors).copy()
            nbr[eid < 0] = -1
            np.testing.assert_array_equal(nbr, want[2])
    assert n_calls > 0


@pytest.mark.parametrize("name", ["k4_mono", "k4_shuffled_t", "k10_mono"])
def test_sampler_oracle_matches_reference(golden, name):
    check_sampler_replay(golden(f"sampler_{name}.npz"), RefLastNeighborLoader)


def test_sampler_reset(golden):
    z = golden("sampler_k4_mono.npz")
    ld = RefLastNeighborLoader(40, 4)
    ld.insert(np.array([1, 2]), np.array([3, 4]), np.array([1.0, 2.0], dtype=np.float32))
    ld.reset_state()
    lo, hi, cur = z["reset_eid_min"].tolist()
    assert ld.e_id.min() == lo and ld.e_id.max() == hi and ld.cur_e_id == cur


def test_blocks_oracle_matches_reference(golden):
    z = golden("blocks.npz")
    got = blocks_ref.block_ids(z["src"], z["dst"], int(z["batch"][0]))
    np.testing.assert_array_equal(got, z["blocks"])
    np.testing.assert_array_equal(blocks_ref.get_block([1, 1, 2, 3, 3, 5], [2, 4, 4, 1, 5, 1]), z["small"])


def test_neg_oracle_replays_reference_rng(golden):
    z = golden("negs.npz")
    torch.manual_seed(int(z["seed"][0]))
    got = negs_ref.sample(torch.from_numpy(z["dst_nodes"]), torch.from_numpy(z["pos"]))
    np.testing.assert_array_equal(got.numpy(), z["neg"])
    assert (z["neg"] != z["pos"]).all()


def test_time_encode_and_predictor(golden):
    z = golden("model.npz")
    te = RefTimeEncode(100)
    np.testing.assert_array_equal(te.w.weight.detach().numpy(), z["te_w"])
    out = te(torch.from_numpy(z["te_t"])).detach().numpy()
    np.testing.assert_array_equal(out, z["te_out"])
    pred = RefEdgePredictor(100, 100)
    sd = {k[len("pred_param_"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("pred_param_")}
    pred.load_state_dict(sd)
    pos, neg = pred(torch.from_numpy(z["pred_hs"]), torch.from_numpy(z["pred_hp"]),
                    torch.from_numpy(z["pred_hn"]), neg_samples=int(z["pred_ns"][0]))
    np.testing.assert_allclose(pos.detach().numpy(), z["pred_pos"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(neg.detach().numpy(), z["pred_neg"], rtol=0, atol=1e-6)


def test_model_parameter_inventory(golden):
    from oracle.tgnn_ref import RefTGNN
    z = golden("model.npz")
    m = RefTGNN(172, 100, 50)
    names = [n for n, _ in m.named_parameters()]
    assert names == list(z["param_names"])
    for n, p in m.named_parameters():
        assert tuple(p.shape) == tuple(z[f"shape_{n}"].tolist())
    assert sum(p.numel() for p in m.parameters() if p.requires_grad) == int(z["n_trainable"][0])


@pytest.mark.parametrize("aggr,updater", [("last", "gru"), ("mean", "gru"), ("last", "rnn")])
def test_tgn_memory_oracle_matches_reference_module(golden, aggr, updater):
    """oracle/tgn_ref.RefTGNMemory against the reference's own TGNMemory (modules/memory_module.py:25-215,
    msg_agg.py, msg_func.py; tests/golden/make_goldens.py capture_tgn_memory): the same parameters, the same
    train batches (memory(n_id), update_state in train order), train(False) (the flush), eval batches —
    every returned memory / last_update row and both buffers after every call, plus the per-node store
    sizes and the src-direction stores' event times in node order.  Pins the module's control flow (store
    layout and order, update-vs-store order, t_rel, the flush); the placeholder scatter / time-encoder
    arithmetic the reference module ran with is the oracle's own restatement (parity unpinned there)."""
    from oracle.tgn_ref import RefTGNMemory
    z = golden(f"tgn_memory_{aggr}_{updater}.npz")
    N, d, D, B, n_train, n_eval = z["meta"].tolist()
    mem = RefTGNMemory(N, d, D, D, aggr=aggr, updater=updater)
    sd = {k[2:].replace("__", "."): torch.from_numpy(z[k]) for k in z.files if k.startswith("p_")}
    missing = mem.load_state_dict(sd, strict=False)
    assert not missing.unexpected_keys and set(missing.missing_keys) <= {"memory", "last_update", "_assoc"}
    mem.train()
    for b in range(n_train + n_eval):
        if b == n_train:
            mem.train(False)
            np.testing.assert_allclose(mem.memory.numpy(), z["flush_memory"], rtol=0, atol=2e-6)
            np.testing.assert_array_equal(mem.last_update.numpy(), z["flush_last_update"])
        s, dd = torch.from_numpy(z["src"][b]), torch.from_numpy(z["dst"][b])
        n_id = torch.cat([s, dd, torch.from_numpy(z["extra"][b])]).unique()
        np.testing.assert_array_equal(n_id.numpy(), z[f"b{b}_nid"])
        with torch.no_grad():
            zz, lu = mem(n_id)
            np.testing.assert_allclose(zz.numpy(), z[f"b{b}_z"], rtol=0, atol=2e-6, err_msg=f"batch {b}")
            np.testing.assert_array_equal(lu.numpy(), z[f"b{b}_lu"])
            mem.update_state(s, dd, torch.from_numpy(z["t"][b]), torch.from_numpy(z["msg"][b]))
        np.testing.assert_allclose(mem.memory.numpy(), z[f"b{b}_memory"], rtol=0, atol=2e-6, err_msg=f"batch {b}")
        np.testing.assert_array_equal(mem.last_update.numpy(), z[f"b{b}_last_update"])
        empty = torch.empty(0)
        st_n = np.array([mem.msg_s_store.get(j, (empty,) * 3)[2].numel() for j in range(N)])
        np.testing.assert_array_equal(st_n, z[f"b{b}_store_s_n"])
        np.testing.assert_array_equal(np.array([mem.msg_d_store.get(j, (empty,) * 3)[2].numel() for j in range(N)]),
                                      z[f"b{b}_store_d_n"])
        got_t = [mem.msg_s_store[j][2].numpy().astype(np.float64) for j in range(N) if j in mem.msg_s_store]
        np.testing.assert_array_equal(np.concatenate(got_t or [np.zeros(0)]), z[f"b{b}_store_s_t"])


def test_tgn_oracle_matches_reference_model_wiring(golden):
    """oracle/tgn_ref.RefTGN + train_step against the reference's own model wiring (make_goldens.py
    capture_tgn_model): pyg_model_utils.py:10-43 getModel / getOptimizer called as written, so
    GraphAttentionEmbedding (modules/emb_module.py:11-29: rel_t = last_update[edge_index[0]] - t, edge_attr =
    [time_enc(rel_t) ‖ msg], time_enc shared with the memory) and LinkPredictor (decoder.py) run as the
    reference composes them, with the reference's LastNeighborLoader, over 4 canonical batches with Adam:
    every output, the loss, every parameter gradient (the shared time encoder's summed over both uses),
    memory and last_update after each batch, nothing resynchronised.  The placeholder TransformerConv /
    scatter / time-encoder arithmetic the reference modules ran with is restated on both sides (parity
    unpinned there); this pins the wiring around it."""
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, train_step
    z = golden("tgn_model_wiring.npz")
    N, d, D, B, nb = z["meta"].tolist()
    ref = RefTGN(N, d, hidden=D, aggr="last", dropout=0.0)
    sd = {k[2:].replace("__", "."): torch.from_numpy(z[k]) for k in z.files if k.startswith("p_")}
    missing = ref.load_state_dict(sd, strict=False)
    assert not missing.unexpected_keys
    assert set(missing.missing_keys) <= {"memory.memory", "memory.last_update", "memory._assoc"}, missing.missing_keys
    opt = torch.optim.Adam(ref.parameters(), lr=float(z["lr"][0]))
    loader = RefLastNeighborLoader(N, 10)
    ev_t = torch.from_numpy(z["t"].reshape(-1).astype(np.float32))
    ev_msg = torch.from_numpy(z["msg"])
    named = dict(ref.named_parameters())
    for b in range(nb):
        sl = slice(b * B, (b + 1) * B)
        src, pos, neg = (torch.from_numpy(z[k][b]) for k in ("src", "dst", "neg"))
        loss, po, no = train_step(ref, opt, loader, ev_t, ev_msg, src, pos, neg, ev_t[sl], ev_msg[sl])
        np.testing.assert_allclose(po.numpy(), z[f"b{b}_pos"], rtol=0, atol=2e-6, err_msg=f"batch {b}")
        np.testing.assert_allclose(no.numpy(), z[f"b{b}_neg"], rtol=0, atol=2e-6, err_msg=f"batch {b}")
        assert abs(loss - float(z[f"b{b}_loss"][0])) < 2e-6, b
        grads = {k[len(f"b{b}_g_"):].replace("__", "."): z[k] for k in z.files if k.startswith(f"b{b}_g_")}
        assert set(grads) == set(named), sorted(set(grads) ^ set(named))
        for name, g in grads.items():
            got = named[name].grad.numpy()
            if name == "gnn.conv.lin_key.bias":   # exactly zero in exact arithmetic (softmax shift invariance)
                wscale = float(np.abs(grads["gnn.conv.lin_key.weight"]).max())
                assert np.abs(got).max() <= 1e-4 * wscale and np.abs(g).max() <= 1e-4 * wscale, b
                continue
            scale = max(float(np.abs(g).max()), 1e-6)
            np.testing.assert_allclose(got, g, rtol=0, atol=2e-5 * scale, err_msg=f"batch {b} {name}")
        np.testing.assert_allclose(ref.memory.memory.detach().numpy(), z[f"b{b}_memory"], rtol=0, atol=2e-6,
                                   err_msg=f"batch {b}")
        np.testing.assert_array_equal(ref.memory.last_update.numpy(), z[f"b{b}_last_update"])
