"""GPU parity of the HIP temporal sampler (tgnx_ring_*) against the reference goldens and the
oracle: bit-exact neighbour indices, e_ids, times, assoc and ring state."""
import numpy as np
import pytest
import torch

from oracle.sampler_ref import RefLastNeighborLoader
from test_oracle_goldens import check_sampler_replay

pytestmark = pytest.mark.gpu


def _gpu_loader_cls():
    from tgnx.sampler import LastNeighborLoader

    def make(N, K):
        return LastNeighborLoader(N, K, device="cuda")
    return make


@pytest.mark.parametrize("name", ["k4_mono", "k4_shuffled_t", "k10_mono"])
def test_hip_sampler_matches_reference_goldens(golden, name):
    check_sampler_replay(golden(f"sampler_{name}.npz"), _gpu_loader_cls())


def _compare(ref, gpu, q):
    a = ref(q)
    b = gpu(torch.from_numpy(q))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(y.cpu().numpy(), x)
    np.testing.assert_array_equal(gpu._assoc.cpu().numpy()[a[0]], ref._assoc[a[0]])


@pytest.mark.parametrize("N,K,B,nb,monotone,dup", [
    (9227, 10, 200, 12, True, False),      # wiki-shaped ids, batch 200
    (500, 10, 600, 6, True, False),        # many collisions (> K entries per node): canonical rule
    (50_000, 4, 2000, 4, False, True),     # non-monotone times, duplicate query ids
    (1_000_000, 10, 600, 3, True, False),  # comment-sized id space (bitmap of 1M nodes)
])
def test_hip_sampler_random_streams_vs_oracle(N, K, B, nb, monotone, dup):
    from tgnx.sampler import LastNeighborLoader
    rng = np.random.default_rng(N + K + B)
    ref = RefLastNeighborLoader(N, K)
    gpu = LastNeighborLoader(N, K, device="cuda")
    t0 = 0.0
    pool = rng.integers(0, N, size=max(64, N // 50))
    for _ in range(nb):
        src = rng.choice(pool, size=B)
        dst = rng.choice(pool, size=B)
        if monotone:
            t = (t0 + np.sort(rng.integers(0, 1000, size=B))).astype(np.float32)
            t0 = float(t.max())
        else:
            t = rng.integers(0, 10**6, size=B).astype(np.float32)
        q = np.unique(np.concatenate([src, dst, rng.integers(0, N, size=B)]))
        if dup:
            q = np.concatenate([q, q[: len(q) // 3]])
        _compare(ref, gpu, q)
        ref.insert(src, dst, t)
        gpu.insert(torch.from_numpy(src), torch.from_numpy(dst), torch.from_numpy(t))
        torch.cuda.synchronize()
        eid = gpu.e_id.cpu().numpy()
        np.testing.assert_array_equal(eid, ref.e_id)
        np.testing.assert_array_equal(gpu.t.cpu().numpy(), ref.t)
        nb_ = gpu.neighbors.cpu().numpy()
        np.testing.assert_array_equal(nb_[eid >= 0], ref.neighbors[ref.e_id >= 0])
        touched = np.unique(np.concatenate([src, dst]))
        np.testing.assert_array_equal(gpu._assoc.cpu().numpy()[touched], ref._assoc[touched])


def test_hip_sampler_empty_and_reset():
    from tgnx.sampler import LastNeighborLoader
    gpu = LastNeighborLoader(100, 5, device="cuda")
    nid, ei, eid, t = gpu(torch.tensor([7, 3, 3], dtype=torch.long))
    assert nid.tolist() == [3, 7] and ei.shape == (2, 0) and eid.numel() == 0
    gpu.insert(torch.tensor([1]), torch.tensor([2]), torch.tensor([5.0]))
    nid, ei, eid, t = gpu(torch.tensor([2]))
    assert nid.tolist() == [1, 2] and ei.tolist() == [[0], [1]] and eid.tolist() == [0] and t.tolist() == [5.0]
    gpu.reset_state()
    assert gpu.cur_e_id == 0 and int(gpu.e_id.max()) == -1 and float(gpu.t.max()) == -1.0
    nid, ei, eid, t = gpu(torch.tensor([2]))
    assert nid.tolist() == [2] and eid.numel() == 0


def test_hip_neg_sampler_distribution():
    from tgnx.neg import NegLinkSamplerDest
    dst_nodes = torch.arange(100, 120)
    s = NegLinkSamplerDest(dst_nodes, device="cuda", seed=3)
    pos = torch.full((200_000,), 105, dtype=torch.long)
    neg = s.sample(pos).cpu()
    assert (neg != 105).all()
    assert ((neg >= 100) & (neg < 120)).all()
    cnt = torch.bincount(neg - 100, minlength=20).double()
    expect = 200_000 / 19
    assert cnt[5] == 0
    others = torch.cat([cnt[:5], cnt[6:]])
    assert (others - expect).abs().max() < 6 * expect ** 0.5   # uniform over the 19 others
    neg2 = s.sample(pos).cpu()
    assert not torch.equal(neg, neg2)   # fresh draws per call
