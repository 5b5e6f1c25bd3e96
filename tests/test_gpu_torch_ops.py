"""GPU parity of torch.ops.tgnx (csrc/tgnx_torch.cpp: TORCH_LIBRARY over the C ABI) against the
oracle restatements: the LastNeighborLoader ring (neighbor_loader.py:26-109) bit-exact over a stream of
sample / insert calls, the negative sampler equal to the ctypes path's draw (same counter-based stream),
the t-CSR build and recent sampler bit-exact (oracle/tcsr_ref.py), and the MFMA GEMM against torch fp32."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from tgnx import ops
    return ops.load()


def test_ring_ops_match_oracle():
    from oracle.sampler_ref import RefLastNeighborLoader
    ns = _ops()
    N, K, B = 3000, 10, 300
    dev = torch.device("cuda")
    nbr = torch.full((N, K), -1, dtype=torch.long, device=dev)
    eid = torch.empty((N, K), dtype=torch.long, device=dev)
    t = torch.empty((N, K), dtype=torch.float, device=dev)
    assoc = torch.zeros(N, dtype=torch.long, device=dev)
    ns.ring_reset(eid, t)
    ref = RefLastNeighborLoader(N, K)
    rng = np.random.default_rng(4)
    cur = 0
    for step in range(6):
        src, dst = rng.integers(0, N, B), rng.integers(0, N, B)
        tt = (step * 1000 + np.sort(rng.integers(0, 1000, B))).astype(np.float32)
        q = np.unique(np.concatenate([src, dst, rng.integers(0, N, B)]))
        got = ns.ring_sample(nbr, eid, t, assoc, torch.from_numpy(q).to(dev))
        want = ref(q)
        for g, w in zip(got, want):
            assert np.array_equal(g.cpu().numpy(), w), step
        ns.ring_insert(nbr, eid, t, torch.from_numpy(src).to(dev), torch.from_numpy(dst).to(dev),
                       torch.from_numpy(tt).to(dev), cur, assoc)
        ref.insert(src, dst, tt)
        cur += B
        assert np.array_equal(eid.cpu().numpy(), ref.e_id), step
        assert np.array_equal(t.cpu().numpy(), ref.t), step


def test_neg_sample_op_equals_ctypes_path():
    from tgnx.neg import NegLinkSamplerDest
    ns = _ops()
    dst_nodes = torch.arange(100, 1100)
    pos = torch.randint(100, 1100, (5000,))
    s = NegLinkSamplerDest(dst_nodes, device="cuda", seed=7)
    a = s.sample(pos)
    b = ns.neg_sample(dst_nodes.cuda(), pos.cuda(), 7, 0)
    assert torch.equal(a, b)
    assert not bool((b == pos.cuda()).any())


def test_tcsr_ops_match_oracle():
    from oracle.tcsr_ref import gen_graph, sample_recent
    ns = _ops()
    rng = np.random.default_rng(1)
    N, E, K = 1500, 20000, 10
    src, dst = rng.integers(0, N, E), rng.integers(0, N, E)
    tt = np.sort(rng.integers(0, 10 * E, E)).astype(np.float32)
    ip, ix, ei, ts, chrono = ns.tcsr_build(torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda(),
                                           torch.from_numpy(tt).cuda(), N, True)
    rip, rix, rei, rts = gen_graph(src, dst, tt, N)
    assert chrono
    for g, w in ((ip, rip), (ix, rix), (ei, rei), (ts, rts)):
        assert np.array_equal(g.cpu().numpy(), w)
    roots = rng.integers(0, N, 700)
    cut = rng.integers(0, E, 700)
    nbr, oe, ot, cnt = ns.tcsr_sample(ip, ix, ei, ts, K, torch.from_numpy(roots).cuda(), 0, torch.from_numpy(cut).cuda())
    wn, we, wt = sample_recent(rip, rix, rei, rts, roots, K, cut_eid=cut)[:3]
    assert np.array_equal(nbr.cpu().numpy(), wn) and np.array_equal(oe.cpu().numpy(), we)
    assert np.array_equal(ot.cpu().numpy(), wt)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_op_matches_torch_fp32(ta, tb):
    ns = _ops()
    g = torch.Generator().manual_seed(0)
    M, N, K = 437, 400, 572
    A = torch.randn((K, M) if ta else (M, K), generator=g).cuda()
    B = torch.randn((N, K) if tb else (K, N), generator=g).cuda()
    bias = torch.randn(N, generator=g).cuda()
    C = ns.gemm_f32(A, B, bias, ta, tb)
    ref = (A.T if ta else A).double() @ (B.T if tb else B).double() + bias.double()
    assert float((C.double() - ref).abs().max() / ref.abs().max()) < 1e-5
