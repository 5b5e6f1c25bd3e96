"""CPU tests of the TGN memory path's host surface (no GPU): the oracle pinned by the reference's own
module outputs (tests/golden/msg.npz: modules/msg_func.py IdentityMessage; tests/golden/link_pred.npz:
modules/decoder.py LinkPredictor), the aggregation semantics the kernels follow, and
the C ABI's host-side entry points (parameter layout against the reference's parameter shapes,
workspace / store sizing, argument rejection)."""
import ctypes

import numpy as np
import pytest
import torch


def test_identity_message_matches_reference(golden):
    from oracle.tgn_ref import identity_message
    z = golden("msg.npz")
    out = identity_message(*(torch.from_numpy(z[k]) for k in ("zs", "zd", "raw", "te")))
    np.testing.assert_array_equal(out.numpy(), z["out"])
    assert out.shape[1] == int(z["out_channels"][0])


def test_link_predictor_matches_reference(golden):
    from oracle.tgn_ref import RefLinkPredictor
    z = golden("link_pred.npz")
    lp = RefLinkPredictor(6)
    sd = {k[2:].replace("__", "."): torch.from_numpy(z[k]) for k in z.files if k.startswith("p_")}
    lp.load_state_dict(sd)
    with torch.no_grad():
        out = lp(torch.from_numpy(z["zs"]), torch.from_numpy(z["zd"]))
    np.testing.assert_allclose(out.numpy(), z["out"], rtol=0, atol=1e-7)


def test_last_aggregator_ties_and_empty_rows():
    """LastAggregator (msg_agg.py:15-21): the message at the max t per node, ties -> the first
    message (torch_scatter CPU), nodes without messages -> zeros; last_update fill 0."""
    from oracle.tgn_ref import last_aggregate, mean_aggregate, scatter_max_first
    msg = torch.arange(12, dtype=torch.float32).view(6, 2)
    idx = torch.tensor([0, 2, 0, 2, 2, 0])
    t = torch.tensor([5, 3, 5, 7, 7, 1])          # node 0: tie at t=5 (rows 0, 2); node 2: tie at 7 (rows 3, 4)
    out = last_aggregate(msg, idx, t, 4)
    np.testing.assert_array_equal(out.numpy(), np.array([[0, 1], [0, 0], [6, 7], [0, 0]], dtype=np.float32))
    mx, arg = scatter_max_first(t, idx, 4)
    np.testing.assert_array_equal(mx.numpy(), [5, 0, 7, 0])
    np.testing.assert_array_equal(arg.numpy(), [0, 6, 3, 6])
    mean = mean_aggregate(msg, idx, t, 4)
    np.testing.assert_allclose(mean.numpy(), [[(0 + 4 + 10) / 3, (1 + 5 + 11) / 3], [0, 0],
                                              [(2 + 6 + 8) / 3, (3 + 7 + 9) / 3], [0, 0]], rtol=1e-6)


def _cfg(N=9227, E=157474, D=100, d=172, B=200, kn=1, aggr=0, heads=2, layers=1, updater=0):
    from tgnx.tgn import TgnConfig
    return TgnConfig(num_nodes=N, num_events=E, ring=10, mem_dim=D, msg_dim=d, heads=heads, max_batch=B, max_neg=kn,
                     aggr=aggr, dropout=0.1, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8, layers=layers,
                     updater=updater)


@pytest.mark.parametrize("updater", ["gru", "rnn"])
@pytest.mark.parametrize("layers", [1, 2])
@pytest.mark.parametrize("D,d", [(100, 172), (100, 1), (32, 16), (6, 2)])
def test_param_layout_matches_reference_shapes(D, d, layers, updater):
    """tgnx_tgn_param_layout: one slot per reference parameter (pyg_model_utils.py:10-36 modules; layers = 2
    adds the oracle's gnn.conv2; the memory updater a GRUCell or an RNNCell, memory_module.py:70-78), sized
    as the reference's shapes, 16-B aligned, disjoint; the projection stride invariant (the same stride
    for conv2)."""
    from oracle.tgn_ref import RefTGN
    from tgnx import _lib
    from tgnx.tgn import PARAM_ORDER, PARAM_ORDER2, param_shapes
    order = PARAM_ORDER2 if layers == 2 else PARAM_ORDER
    cfg = _cfg(D=D, d=d, layers=layers, updater=1 if updater == "rnn" else 0)
    off = (ctypes.c_int64 * (len(order) + 1))()
    _lib.call("tgnx_tgn_param_layout", ctypes.byref(cfg), off)
    off = list(off)
    ref = {k: tuple(v.shape) for k, v in RefTGN(50, d, hidden=D, layers=layers, updater=updater).named_parameters()}
    shapes = param_shapes(D, d, layers, updater)
    assert set(ref) == set(order) and all(ref[k] == shapes[k] for k in order)
    spans = sorted((off[i], off[i] + int(np.prod(shapes[k]))) for i, k in enumerate(order))
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0
    assert all(o % 4 == 0 for o in off[:-1]) and spans[-1][1] <= off[-1]
    o = dict(zip(order, off))
    strides = set()
    for cv in (("conv", "conv2") if layers == 2 else ("conv",)):
        w = [o[f"gnn.{cv}.lin_{k}.weight"] for k in ("query", "key", "value", "skip")]
        b = [o[f"gnn.{cv}.lin_{k}.bias"] for k in ("query", "key", "value", "skip")]
        assert len({y - x for x, y in zip(w, w[1:])}) == 1 and len({y - x for x, y in zip(b, b[1:])}) == 1
        strides.add((w[1] - w[0], b[1] - b[0]))
    assert len(strides) == 1


def test_two_hop_workspace_sizing():
    """layers = 2 sizes the outer sample up to (K + 1)x the 1-hop one; the comment-shaped config (B = 600)
    fits comfortably in one MI355X's HBM."""
    from tgnx import _lib
    L = _lib.lib()
    one = L.tgnx_tgn_ws_bytes(ctypes.byref(_cfg()))
    two = L.tgnx_tgn_ws_bytes(ctypes.byref(_cfg(layers=2)))
    assert two > 2 * one                                   # capped by N = 9,227 here
    comment = _cfg(N=994790, E=44314507, d=2, B=600, kn=1, layers=2)
    assert 0 < L.tgnx_tgn_ws_bytes(ctypes.byref(comment)) < (16 << 30)
    bad = _cfg(layers=3)
    assert L.tgnx_tgn_ws_bytes(ctypes.byref(bad)) == 0 and b"layers" in L.tgnx_last_error()


def test_workspace_and_store_sizing():
    from tgnx import _lib
    L = _lib.lib()
    cfg = _cfg()
    assert L.tgnx_tgn_store_words(ctypes.byref(cfg)) == 4 * cfg.num_nodes + 2 * cfg.num_events
    ws1 = L.tgnx_tgn_ws_bytes(ctypes.byref(cfg))
    assert ws1 > 0
    big = _cfg(kn=999)                                        # TGB eval negatives grow the workspace
    assert L.tgnx_tgn_ws_bytes(ctypes.byref(big)) > ws1
    review = _cfg(N=352637, E=4873540, d=1, kn=100, aggr=1)
    assert 0 < L.tgnx_tgn_ws_bytes(ctypes.byref(review)) < (8 << 30)


@pytest.mark.parametrize("field,value,msg", [("heads", 8, b"heads"), ("mem_dim", 101, b"mem_dim"),
                                             ("max_batch", 5000, b"max_batch"), ("aggr", 3, b"aggr"),
                                             ("ring", 0, b"ring"), ("updater", 2, b"updater")])
def test_config_rejections(field, value, msg):
    from tgnx import _lib
    L = _lib.lib()
    cfg = _cfg()
    setattr(cfg, field, value)
    assert L.tgnx_tgn_ws_bytes(ctypes.byref(cfg)) == 0
    off = (ctypes.c_int64 * 22)()
    assert L.tgnx_tgn_param_layout(ctypes.byref(cfg), off) != 0
    assert msg in L.tgnx_last_error()


def test_two_hop_oracle_reduces_to_one_hop():
    """The 2-hop extension (oracle RefTGN(layers=2)): with conv2 the identity (value weights 0, skip = I)
    the 2-hop scores equal the 1-hop model's on the same stream — the 2-hop node set, assoc and the
    layer-1 outputs of the roots are consistent with the 1-hop path."""
    from oracle.sampler_ref import RefLastNeighborLoader
    from oracle.tgn_ref import RefTGN, eval_step, train_step
    torch.manual_seed(0)
    N, d, D, B = 60, 5, 8, 16
    rng = np.random.default_rng(0)
    E = 6 * B
    src, dst = torch.from_numpy(rng.integers(0, N, E)), torch.from_numpy(rng.integers(0, N, E))
    t = torch.from_numpy(np.sort(rng.random(E) * 100).astype(np.float32))
    msg = torch.randn(E, d)
    m1 = RefTGN(N, d, hidden=D, dropout=0.0)
    m2 = RefTGN(N, d, hidden=D, dropout=0.0, layers=2)
    sd = m1.state_dict()
    with torch.no_grad():
        for k, v in m2.state_dict().items():
            if k in sd:
                v.copy_(sd[k])
        c2 = m2.gnn.conv2
        for lin in (c2.lin_query, c2.lin_key, c2.lin_value, c2.lin_edge):
            lin.weight.zero_()
            if lin.bias is not None:
                lin.bias.zero_()
        c2.lin_skip.weight.copy_(torch.eye(D))
        c2.lin_skip.bias.zero_()
    l1, l2 = RefLastNeighborLoader(N, 3), RefLastNeighborLoader(N, 3)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.0)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.0)
    for b in range(E // B - 1):
        sl = slice(b * B, (b + 1) * B)
        neg = torch.from_numpy(rng.integers(0, N, B))
        a = train_step(m1, o1, l1, t, msg, src[sl], dst[sl], neg, t[sl], msg[sl])
        c = train_step(m2, o2, l2, t, msg, src[sl], dst[sl], neg, t[sl], msg[sl])
        torch.testing.assert_close(a[1], c[1], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(a[2], c[2], rtol=1e-5, atol=1e-6)
    sl = slice(E - B, E)
    negs = torch.from_numpy(rng.integers(0, N, (B, 4)))
    a = eval_step(m1, l1, t, msg, src[sl], dst[sl], negs, t[sl], msg[sl])
    c = eval_step(m2, l2, t, msg, src[sl], dst[sl], negs, t[sl], msg[sl])
    torch.testing.assert_close(a[1], c[1], rtol=1e-5, atol=1e-6)


def test_dyrep_model_surface():
    """DyRepMemory (modules/memory_module.py:218-421) behind getModel: memory_updater_type 'gru' | 'rnn' with
    the reference's state-dict names (memory.memory_updater.*, shared with TGNMemory, :70-78); embeddings in
    an unknown updater rejected as the reference does (:75-78); embedding messages only on DyRepMemory, 1 hop."""
    from oracle.tgn_ref import RefTGN
    from tgnx.tgn import PARAM_ORDER, param_shapes
    ref = RefTGN(30, 4, hidden=8, updater="rnn")
    assert isinstance(ref.memory.memory_updater, torch.nn.RNNCell)
    shapes = param_shapes(8, 4, 1, "rnn")
    assert {k: tuple(v.shape) for k, v in ref.named_parameters()} == {k: shapes[k] for k in PARAM_ORDER}
    assert shapes["memory.memory_updater.weight_ih"] == (8, 3 * 8 + 4)
    from tgnx.tgn import TGNModel
    with pytest.raises(ValueError):
        TGNModel(30, 10, 4, 8, "cpu", memory="tgn", updater="rnn", use_dst_emb_in_msg=True)
    with pytest.raises(NotImplementedError):
        TGNModel(30, 10, 4, 8, "cpu", memory="dyrep", updater="rnn", layers=2, use_dst_emb_in_msg=True)
    with pytest.raises(ValueError):
        TGNModel(30, 10, 4, 8, "cpu", memory="dyrep", updater="lstm")


def test_dyrep_embedding_messages_follow_the_reference_loop():
    """oracle RefTGNMemory._compute_msg with embeddings (vectorised isin) against the reference's own per-entry
    loop (memory_module.py:387-408, restated literally here: `if s in n_id` per stored message), on stores
    filled by two batches: the source / destination memory rows replaced by embeddings[assoc[node]] exactly
    for the endpoints in n_id."""
    from oracle.tgn_ref import RefTGNMemory
    torch.manual_seed(0)
    N, d, D = 40, 3, 6
    for flags in ((1, 0), (0, 1), (1, 1)):
        mem = RefTGNMemory(N, d, D, D, "last", "rnn", *flags)
        mem.memory.copy_(torch.randn(N, D))
        g = torch.Generator().manual_seed(1)
        for b in range(2):
            src, dst = torch.randint(0, N, (12,), generator=g), torch.randint(0, N, (12,), generator=g)
            t = torch.arange(12, dtype=torch.float32) + 20 * b
            mem._update_msg_store(src, dst, t, torch.randn(12, d), mem.msg_s_store)
            mem._update_msg_store(dst, src, t, torch.randn(12, d), mem.msg_d_store)
        n_id = torch.cat([src, dst]).unique()
        emb = torch.randn(N, D)
        assoc = torch.randperm(N)
        inv = torch.empty(N, dtype=torch.long)
        inv[assoc] = torch.arange(N)
        embeddings = emb[inv]                       # embeddings[assoc[v]] == emb[v]
        for store in (mem.msg_s_store, mem.msg_d_store):
            msg, _, s_, d_ = mem._compute_msg(n_id, store, embeddings, assoc)
            src_mem, dst_mem = mem.memory[s_].clone(), mem.memory[d_].clone()
            for i, v in enumerate(s_):              # memory_module.py:389-397
                if flags[0] and v in n_id:
                    src_mem[i] = embeddings[assoc[v]]
            for i, v in enumerate(d_):              # :400-408
                if flags[1] and v in n_id:
                    dst_mem[i] = embeddings[assoc[v]]
            assert torch.equal(msg[:, :D], src_mem) and torch.equal(msg[:, D:2 * D], dst_mem)


def test_oracle_epoch_noise_floor_by_time_scale():
    """The premise of tests/test_gpu_tgn_epochs.py (oracle on one thread: torch's multi-threaded CPU scatter
    reductions are not run-to-run deterministic): on a wiki-shaped stream whose timestamps span 2,000 s the
    oracle's 2-epoch trajectory is insensitive to a 1-ulp change of the time-encoder weight (loss sums to 1e-6,
    val MRR exactly), while at the wiki time scale (2,678,373 s) the same change moves the loss sums by 1e-4 or
    more and the epoch-2 val MRR by a visible amount — multi-epoch parity there can only be statistical
    (DESIGN §7)."""
    from epoch_parity import initial_state, oracle_epochs, scaled_stream
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        s = scaled_stream(0, t_max=2000)
        sd = initial_state(s, 0)
        a = oracle_epochs(s, sd, 0)
        assert oracle_epochs(s, sd, 0) == a                      # deterministic on one thread
        b = oracle_epochs(s, sd, 0, perturb="memory.time_enc.lin.weight")
        for e in range(2):
            assert abs(a["loss"][e] - b["loss"][e]) <= 1e-6 * a["loss"][e]
            assert a["mrr"][e] == b["mrr"][e]
        s = scaled_stream(0)
        sd = initial_state(s, 0)
        a = oracle_epochs(s, sd, 0)
        b = oracle_epochs(s, sd, 0, perturb="memory.time_enc.lin.weight")
        for e in range(2):
            assert abs(a["loss"][e] - b["loss"][e]) > 1e-4 * a["loss"][e]
        assert abs(a["mrr"][1] - b["mrr"][1]) > 1e-3
    finally:
        torch.set_num_threads(nt)
