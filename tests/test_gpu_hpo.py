"""Row P at the learning level on the GPU: one seed of the reference's HPO trial-31 configuration
(train.py's PPO on 8 HoverEnv + RateControlWrapper envs, batch 128, 20 epochs, 10 deterministic
evaluations every 50,000 env steps; tests/hpo_repro.py) through the product path -- QuadVecEnv's
HIP env kernels, quad_rollout, quad_ppo_grad, quad_clip_adam -- in a few seconds. Learning is a
chaotic function of every bit, so the bar is the outcome band, not a curve: the last five
evaluations average above 300 (every seed of the committed record is above 380; the reference's last
five are 399-477) and the first is below 100 (the untrained policy crashes within 100 steps).
"""
import pytest

pytestmark = pytest.mark.gpu


def test_hpo_trial31_config_learns_on_the_gpu_path():
    from hpo_repro import run_gpu
    r = run_gpu(0)  # raises unless the fused HIP rollout and learner run
    c = r["curve"]
    assert len(c) == 10 and r["updates"] == 61 and r["optimizer_steps"] == 61 * 64 * 20
    assert c[0] < 100.0
    assert sum(c[5:]) / 5 > 300.0, c
