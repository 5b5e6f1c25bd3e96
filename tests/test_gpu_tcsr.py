"""GPU parity of the t-CSR graph and recent sampler (tgnx_tcsr_build / tgnx_tcsr_sample) — bit-exact:
  * device build == the oracle's gen_graph restatement (oracle/tcsr_ref.py);
  * device sampling == oracle sampling, event-id and TGL time cutoffs, incl. a 10,000-entry hub row
    (several 64-ary search rounds) and roots without entries;
  * event-id cutoff at each batch start == the reference's golden LastNeighborLoader ring states
    (tests/golden/sampler_*.npz) and == the device ring (tgnx_ring_insert) over a wiki-shaped stream."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _build(src, dst, t, N):
    from tgnx.tcsr import TCSR
    return TCSR.build(torch.from_numpy(np.asarray(src)), torch.from_numpy(np.asarray(dst)),
                      torch.from_numpy(np.asarray(t, np.float32)), N, device="cuda")


def _stream(N=2000, E=30000, hub=True, seed=0):
    rng = np.random.default_rng(seed)
    src, dst = rng.integers(0, N, E), rng.integers(0, N, E)
    if hub:
        src[rng.random(E) < 0.33] = 7          # node 7: ~10,000 entries
    t = np.sort(rng.integers(0, 10 * E, E)).astype(np.float32)
    return src, dst, t


def test_build_matches_oracle():
    from oracle.tcsr_ref import gen_graph
    src, dst, t = _stream()
    N = 2000
    g = _build(src, dst, t, N)
    ip, ix, ei, ts = gen_graph(src, dst, t, N)
    assert g.chronological
    np.testing.assert_array_equal(g.indptr.cpu().numpy(), ip)
    np.testing.assert_array_equal(g.eid.cpu().numpy(), ei)
    np.testing.assert_array_equal(g.indices.cpu().numpy(), ix)
    np.testing.assert_array_equal(g.ts.cpu().numpy(), ts)
    assert ip[8] - ip[7] > 9000


@pytest.mark.parametrize("K", [1, 10, 16, 17, 32, 64, 100])   # (<= 16 / <= 32: the grouped kernel; more: a wave per root)
def test_sample_matches_oracle_both_cutoffs(K):
    from oracle.tcsr_ref import gen_graph, sample_recent
    src, dst, t = _stream(seed=1)
    N = 2000
    g = _build(src, dst, t, N)
    ref = gen_graph(src, dst, t, N)
    rng = np.random.default_rng(2)
    roots = np.concatenate([rng.integers(0, N, 3000), [7, 7, 7]])
    cut = rng.integers(0, src.shape[0] + 1, roots.shape[0])
    cut[-3:] = [0, 15000, src.shape[0]]
    got = [x.cpu().numpy() for x in g.sample_recent(torch.from_numpy(roots), K, cut_eid=torch.from_numpy(cut))]
    want = sample_recent(*ref, roots, K, cut_eid=cut)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    ct = rng.integers(0, 10 * src.shape[0], roots.shape[0]).astype(np.float32)
    got = [x.cpu().numpy() for x in g.sample_recent(torch.from_numpy(roots), K, cut_t=torch.from_numpy(ct))]
    want = sample_recent(*ref, roots, K, cut_t=ct)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    got = [x.cpu().numpy() for x in g.sample_recent(torch.from_numpy(roots), K, cut_eid=12345)]
    want = sample_recent(*ref, roots, K, cut_eid=12345)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("name", ["k4_mono", "k10_mono"])
def test_eid_cutoff_equals_reference_ring_goldens(golden, name):
    z = golden(f"sampler_{name}.npz")
    N, K, nb, B, _ = z["meta"].tolist()
    g = _build(z["ins_src"], z["ins_dst"], z["ins_t"], N)
    for bi in range(nb):
        nbr, eid, ts, _ = g.sample_recent(torch.arange(N), K, cut_eid=B * (bi + 1))
        np.testing.assert_array_equal(eid.cpu().numpy(), z["state_eid"][bi])
        np.testing.assert_array_equal(nbr.cpu().numpy(), z["state_nbr"][bi])
        np.testing.assert_array_equal(ts.cpu().numpy(), z["state_t"][bi])


def test_eid_cutoff_equals_device_ring():
    from tgnx.sampler import LastNeighborLoader
    from tgnx.synth import make_stream
    s = make_stream("tgbl-wiki", seed=4, num_events=12000, num_nodes=3000, msg_dim=4)
    N, K, B = s.shape.num_nodes, 10, 200
    g = _build(s.src, s.dst, s.t.astype(np.float32), N)
    ring = LastNeighborLoader(N, K, device="cuda")
    for b0 in range(0, 12000, B):
        if b0 % 2000 == 0:
            nbr, eid, ts, _ = g.sample_recent(torch.arange(N), K, cut_eid=b0)
            e = ring.e_id.cpu().numpy()
            assert np.array_equal(eid.cpu().numpy(), e), b0
            rn = ring.neighbors.cpu().numpy().copy()
            rn[e < 0] = -1
            assert np.array_equal(nbr.cpu().numpy(), rn), b0
            assert np.array_equal(ts.cpu().numpy(), ring.t.cpu().numpy()), b0
        sl = slice(b0, b0 + B)
        ring.insert(torch.from_numpy(s.src[sl]), torch.from_numpy(s.dst[sl]),
                    torch.from_numpy(s.t[sl].astype(np.float32)))
