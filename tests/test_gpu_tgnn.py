"""GPU parity of the fused TGNN step (tgnx_tgnn_*) against the oracle's faithful per-block loop.

Tolerances (fp32; the HIP path reassociates sums — collapsed head dots, online softmax,
slab reductions):  logits and loss rel 2e-4 of the batch's max |value|; gradients rel 2e-3
of the tensor's max |grad|; parameters after Adam abs 2e-6 where the gradient is above the
fp32 cancellation floor (1e-3 of the tensor max), else within ~2 lr per step; ring state, time_assoc bit-exact.
"""
import numpy as np
import pytest

from parity_harness import Pair, rel_err

pytestmark = pytest.mark.gpu


def grad_tol(name):
    # attn_r only reaches the loss through er, which shifts every score of a destination's
    # softmax equally: its gradient is zero except at LeakyReLU kinks, so what remains is a
    # cancellation residue of terms ~1e2x larger — compare it at the cancelled scale.
    return 5e-2 if name.endswith("attn_r") else 2e-3


@pytest.fixture(scope="module")
def pair():
    return Pair(N=400, E=1800, d=172, B=200, Kn_eval=20, seed=0)


def test_train_steps_match_oracle(pair):
    for step in range(4):
        if step:
            pair.sync_from_ref()
        r = pair.train_step()
        assert rel_err(r["pos"], r["ref_pos"]) < 2e-4, step
        assert rel_err(r["neg"], r["ref_neg"]) < 2e-4, step
        assert abs(r["loss"] - r["ref_loss"]) < 2e-4 * max(1.0, abs(r["ref_loss"])), step
        rg, gg = pair.ref_grads(), pair.gpu_grads()
        for k, v in rg.items():
            assert rel_err(gg[k], v) < grad_tol(k), (step, k, rel_err(gg[k], v))
        well, allv = pair.param_diff()
        assert max(well.values()) < 2e-6, (step, well)
        assert max(allv.values()) < 2.5e-4, (step, allv)
        ring_ok, ta_ok = pair.state_equal()
        assert ring_ok and ta_ok, step


def test_eval_steps_match_oracle(pair):
    pair.sync_from_ref()
    for step in range(2):
        r = pair.eval_step(quirk=True)
        assert rel_err(r["pos"], r["ref_pos"]) < 2e-4
        assert rel_err(r["neg"], r["ref_neg"]) < 2e-4
        assert abs(r["mrr"] - r["ref_mrr"]) < 1e-3
        ring_ok, ta_ok = pair.state_equal()
        assert ring_ok and ta_ok


def test_train_after_eval_matches_oracle(pair):
    # eval left time_assoc = max(last block) everywhere (model_utils.py:77-79); train must see it
    pair.sync_from_ref()
    r = pair.train_step()
    assert rel_err(r["pos"], r["ref_pos"]) < 2e-4
    rg, gg = pair.ref_grads(), pair.gpu_grads()
    for k, v in rg.items():
        assert rel_err(gg[k], v) < grad_tol(k), k


def test_small_feature_dim_and_small_times():
    # review/coin-shaped edge features (d=1) exercise the one-dim-per-lane path
    p = Pair(N=300, E=900, d=1, B=150, Kn_eval=8, seed=3, t_max=5000)
    for _ in range(3):
        r = p.train_step()
        assert rel_err(r["pos"], r["ref_pos"]) < 2e-4
        rg, gg = p.ref_grads(), p.gpu_grads()
        for k, v in rg.items():
            assert rel_err(gg[k], v) < grad_tol(k), k
    r = p.eval_step(quirk=False)
    assert rel_err(r["neg"], r["ref_neg"]) < 1.0  # ref uses the tile pairing; only shapes/finite here
    assert np.isfinite(r["neg"]).all()


def test_multi_step_trajectory_small_time_scale():
    # no re-sync: at small time scales the whole trajectory (params, Adam moments, state) must agree
    p = Pair(N=350, E=1600, d=172, B=200, Kn_eval=10, seed=5, t_max=5000)
    for step in range(6):
        r = p.train_step()
        assert rel_err(r["pos"], r["ref_pos"]) < 1e-3, step
        assert rel_err(r["neg"], r["ref_neg"]) < 1e-3, step
        assert all(p.state_equal()), step
    well, _ = p.param_diff()
    assert max(well.values()) < 1e-5, well
    r = p.eval_step()
    assert abs(r["mrr"] - r["ref_mrr"]) < 5e-3
