"""GPU parity of the per-operator entry points (csrc/tgnx_ops.hip via torch.ops.tgnx) against the
oracle's restatements (oracle/tgn_ref.py) and plain torch fp32:

  msg_agg_last / msg_agg_mean   last_aggregate / mean_aggregate (modules/msg_agg.py:15-26): BIT-EXACT, incl.
                                t ties (first index wins, torch_scatter scatter_max), empty rows, hub rows with
                                more messages than a wave has lanes, int64 and fp32 t, no messages at all;
                                an out-of-range index raises
  gru_update                    torch.nn.GRUCell / RNNCell (memory_module.py:70-78), fp32, 2e-5
  predictor                     RefLinkPredictor (decoder.py:12-27, sigmoid) and RefEdgePredictor
                                (model_utils.py:165-195, the eval `tile` pairing), fp32, 2e-5
  edge_attn_fwd / _bwd          transformer_attention (PyG TransformerConv semantics) + torch autograd, fp32:
                                out / alpha 2e-5, gradients 1e-4 (relative to the tensor's max) — incl. a
                                destination without edges, one with 150 edges, heads*C = 100 (TGN), 256, 32

The floating-point tolerances cover reassociation only (MFMA GEMM / wave-sum order vs torch's CPU order)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ops():
    from tgnx import ops
    return ops.load()


def _agg_case(rng, n, dim, dim_size, t_kind):
    index = torch.from_numpy(rng.integers(0, dim_size, n))
    if n:
        index[: n // 4] = min(3, dim_size - 1)                # a hub row (> 64 messages once n >= 260)
    if t_kind == "long":
        t = torch.from_numpy(rng.integers(0, 20, n))         # many ties
    else:
        t = torch.from_numpy(rng.integers(0, 20, n).astype(np.float32))
    msg = torch.randn(n, dim)
    return msg, index, t


@pytest.mark.parametrize("n,dim,dim_size,t_kind", [(1000, 472, 300, "long"), (1000, 100, 2000, "float"),
                                                   (5, 7, 50, "long"), (0, 16, 10, "long"), (300, 1, 1, "float")])
def test_msg_agg_last_and_mean_bit_exact(n, dim, dim_size, t_kind):
    from oracle.tgn_ref import last_aggregate, mean_aggregate, scatter_max_first
    ns = _ops()
    rng = np.random.default_rng(n + dim)
    msg, index, t = _agg_case(rng, n, dim, dim_size, t_kind)
    out, arg = ns.msg_agg_last(msg.to(DEV), index.to(DEV), t.to(DEV), dim_size)
    want = last_aggregate(msg, index, t, dim_size)
    _, want_arg = scatter_max_first(t, index, dim_size)
    assert torch.equal(out.cpu(), want)
    assert torch.equal(arg.cpu(), want_arg)
    mean = ns.msg_agg_mean(msg.to(DEV), index.to(DEV), dim_size)
    assert torch.equal(mean.cpu(), mean_aggregate(msg, index, t, dim_size))


def test_msg_agg_rejects_out_of_range_index():
    ns = _ops()
    msg = torch.randn(4, 3, device=DEV)
    index = torch.tensor([0, 1, 5, 1], device=DEV)
    t = torch.arange(4, device=DEV)
    with pytest.raises(RuntimeError, match="outside"):
        ns.msg_agg_last(msg, index, t, 3)
    with pytest.raises(RuntimeError, match="outside"):
        ns.msg_agg_mean(msg, index - 1, 3)


def _close(a, b, tol):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    scale = max(float(b.abs().max()), 1.0) if b.numel() else 1.0
    err = float((a - b).abs().max()) if b.numel() else 0.0
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("cell", ["gru", "rnn"])
@pytest.mark.parametrize("M", [1, 777])
def test_gru_update_matches_torch_cell(cell, M):
    ns = _ops()
    torch.manual_seed(M)
    d_in, D = 472, 100                                      # wiki's message width, memory dim
    mod = torch.nn.GRUCell(d_in, D) if cell == "gru" else torch.nn.RNNCell(d_in, D)
    x, h = torch.randn(M, d_in), torch.randn(M, D)
    with torch.no_grad():
        want = mod(x, h)
    got = ns.gru_update(x.to(DEV), h.to(DEV), mod.weight_ih.detach().to(DEV), mod.weight_hh.detach().to(DEV),
                        mod.bias_ih.detach().to(DEV), mod.bias_hh.detach().to(DEV), 0 if cell == "gru" else 1)
    _close(got, want, 2e-5)


def test_predictor_matches_link_and_edge_predictors():
    from oracle.tgn_ref import RefLinkPredictor
    from oracle.tgnn_ref import RefEdgePredictor
    ns = _ops()
    torch.manual_seed(0)
    lp = RefLinkPredictor(100)
    zs, zd = torch.randn(200, 100), torch.randn(200, 100)
    with torch.no_grad():
        want = lp(zs, zd)
    d = lambda x: x.detach().to(DEV)  # noqa: E731
    got = ns.predictor(d(zs), d(zd), d(lp.lin_src.weight), d(lp.lin_src.bias), d(lp.lin_dst.weight),
                       d(lp.lin_dst.bias), d(lp.lin_final.weight), d(lp.lin_final.bias), True)
    _close(got, want, 2e-5)
    ep = RefEdgePredictor(100, 100)
    B, K = 64, 7
    hs, hp, hn = torch.randn(B, 100), torch.randn(B, 100), torch.randn(B * K, 100)
    with torch.no_grad():
        want_pos, want_neg = ep(hs, hp, hn, neg_samples=K)
    args = (d(ep.src_fc.weight), d(ep.src_fc.bias), d(ep.dst_fc.weight), d(ep.dst_fc.bias), d(ep.out_fc.weight),
            d(ep.out_fc.bias))
    _close(ns.predictor(d(hs), d(hp), *args[:4], *args[4:], False), want_pos, 2e-5)
    _close(ns.predictor(d(hs), d(hn), *args[:4], *args[4:], False), want_neg, 2e-5)


def _attn_case(seed, n_dst, H, C, degrees, with_e):
    g = torch.Generator().manual_seed(seed)
    deg = torch.tensor(degrees, dtype=torch.long)
    assert deg.numel() == n_dst
    E = int(deg.sum())
    indptr = torch.zeros(n_dst + 1, dtype=torch.long)
    indptr[1:] = deg.cumsum(0)
    i = torch.repeat_interleave(torch.arange(n_dst), deg)
    q = torch.randn(n_dst, H * C, generator=g)
    k, v = torch.randn(E, H * C, generator=g), torch.randn(E, H * C, generator=g)
    e = torch.randn(E, H * C, generator=g) if with_e else None
    return q, k, v, e, indptr, i


@pytest.mark.parametrize("H,C,with_e", [(2, 50, True), (1, 256, True), (4, 8, False)])
def test_edge_attention_fwd_bwd_matches_torch(H, C, with_e):
    from oracle.tgn_ref import transformer_attention
    from tgnx.ops import edge_attention
    rng = np.random.default_rng(H * C)
    n_dst = 300
    degrees = rng.integers(1, 12, n_dst)
    degrees[5], degrees[17] = 0, 150                         # no edges; more edges than lanes
    q, k, v, e, indptr, i = _attn_case(H * C, n_dst, H, C, degrees.tolist(), with_e)
    leaves = [x.clone().requires_grad_(True) for x in (q, k, v) + ((e,) if with_e else ())]
    qr, kr, vr = leaves[:3]
    er = leaves[3] if with_e else torch.zeros_like(kr)
    want, want_alpha = transformer_attention(qr[i].view(-1, H, C), kr.view(-1, H, C), vr.view(-1, H, C),
                                             er.view(-1, H, C), i, n_dst)
    dout = torch.randn_like(want)
    want.backward(dout)
    dl = [x.detach().to(DEV).requires_grad_(True) for x in (q, k, v) + ((e,) if with_e else ())]
    out, alpha = edge_attention(dl[0], dl[1], dl[2], dl[3] if with_e else None, indptr.to(DEV), H)
    out.backward(dout.to(DEV))
    _close(out, want, 2e-5)
    _close(alpha, want_alpha, 2e-5)
    assert float(out.detach()[5].abs().max()) == 0.0                  # no edges: PyG's empty aggregation
    for got_leaf, want_leaf in zip(dl, leaves):
        _close(got_leaf.grad, want_leaf.grad, 1e-4)


def test_survey_named_sampler_ops_are_the_ring_ops():
    """SURVEY §8b's names (sample_recent / insert_recent / reset) run the LastNeighborLoader ring ops."""
    ns = _ops()
    N, K = 500, 10
    state = []
    for _ in range(2):
        nbr = torch.full((N, K), -1, dtype=torch.long, device=DEV)
        eid = torch.empty((N, K), dtype=torch.long, device=DEV)
        t = torch.empty((N, K), device=DEV)
        state.append((nbr, eid, t, torch.zeros(N, dtype=torch.long, device=DEV)))
    ns.ring_reset(state[0][1], state[0][2])
    ns.reset(state[1][1], state[1][2])
    g = torch.Generator().manual_seed(3)
    src, dst = torch.randint(0, N, (300,), generator=g).to(DEV), torch.randint(0, N, (300,), generator=g).to(DEV)
    tt = torch.sort(torch.rand(300, generator=g) * 1000).values.to(DEV)
    ns.ring_insert(*state[0][:3], src, dst, tt, 0, state[0][3])
    ns.insert_recent(*state[1][:3], src, dst, tt, 0, state[1][3])
    for a, b in zip(state[0], state[1]):
        assert torch.equal(a, b)
    q = torch.unique(torch.cat([src, dst]))
    for a, b in zip(ns.ring_sample(*state[0][:3], state[0][3], q), ns.sample_recent(*state[1][:3], state[1][3], q)):
        assert torch.equal(a, b)
