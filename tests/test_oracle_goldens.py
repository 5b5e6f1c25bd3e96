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
