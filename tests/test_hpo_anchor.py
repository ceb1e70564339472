"""Row P at the learning level: the reference's HPO trial 31 (tests/golden/hpo_trial31.json, written
by tools/extract_hpo_curve.py from /root/reference/optuna_full.db) and the reproduction record of
tests/hpo_repro.py (profiles/r06/hpo_repro.json).

CPU-only checks: the fixture's parameters are train.py:50-68's hyperparameters (PPOConfig's
defaults); the harness trains with exactly those; the committed reproduction summary meets the bar
the round-5 verdict set -- every seed's 10-point curve for both paths, the GPU and CPU paths' curves
agreeing within seed spread, and the median final evaluation in the reference's last-five band.
The GPU run of the harness itself is tests/test_gpu_hpo.py.
"""
import json
import os

import numpy as np
import pytest

from hpo_repro import load_anchor, ppo_config, summarize

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORD = os.path.join(REPO, "profiles", "r06", "hpo_repro.json")


def test_fixture_is_train_py_hyperparameters():
    from uav_reinforcement_learning_control_amd.ppo import PPOConfig
    a = load_anchor()
    p, d = a["params"], PPOConfig()
    assert p["learning_rate"] == d.learning_rate and p["clip_range"] == d.clip_range
    assert p["ent_coef"] == d.ent_coef and p["gae_lambda"] == d.gae_lambda
    assert a["user_attrs"]["gamma"] == d.gamma == 1.0 - p["gamma_inv"]
    assert (p["n_steps"], p["batch_size"], p["n_epochs"]) == (d.n_steps, 128, d.n_epochs)
    assert p["net_arch"] == "small" and tuple(d.net_arch) == (128, 128) and p["activation_fn"] == "relu"
    assert a["eval_timesteps"] == [50_000 * (k + 1) for k in range(10)]
    assert len(a["eval_mean_reward"]) == 10 and a["eval_mean_reward"][-1] == a["final_value"]
    assert a["run"]["wrapper"] == "RateControlWrapper" and a["run"]["n_envs"] == 8


def test_harness_config_is_the_trial():
    from uav_reinforcement_learning_control_amd.ppo import PPOConfig
    c, d = ppo_config(), PPOConfig()
    assert c.batch_size == 128 and c.n_steps == 1024 and c.n_epochs == 20
    for k in ("learning_rate", "gamma", "gae_lambda", "clip_range", "ent_coef", "vf_coef", "max_grad_norm",
              "adam_eps", "net_arch", "normalize_advantage"):
        assert getattr(c, k) == getattr(d, k), k
    # SB3's batch clamp (optimize.py:135-144) keeps 128: the 8 x 1024 buffer divides into 64 minibatches
    assert (8 * c.n_steps) % c.batch_size == 0


def test_summary_statistics():
    rng = np.random.default_rng(0)
    base = np.array(load_anchor()["eval_mean_reward"])
    mk = lambda s: {"seed": s, "curve": list(base - 20 + rng.normal(0, 5, 10)), "seconds": 1.0, "train_seconds": 0.5,
                    "optimizer_steps": 1, "env_steps": 1}
    out = summarize({"gpu": [mk(s) for s in range(4)], "cpu": [mk(s) for s in range(4)]})
    assert out["gpu"]["median_final_in_band"] and out["cpu"]["median_final_in_band"]
    assert len(out["gpu_vs_cpu"]["within_2se"]) == 10


@pytest.mark.skipif(not os.path.exists(RECORD), reason="no reproduction record")
def test_reproduction_record():
    r = json.load(open(RECORD))
    band = r["reference"]["band_last5"]
    assert band == [min(r["reference"]["eval_mean_reward"][5:]), max(r["reference"]["eval_mean_reward"][5:])]
    for path in ("gpu", "cpu"):
        p = r[path]
        assert len(p["seeds"]) >= 5 and all(len(c) == 10 for c in p["curves"]), path
        assert p["median_final_in_band"] and band[0] <= p["median_final"] <= band[1], path
    # the two paths agree within seed spread: at every evaluation the mean difference is within two
    # standard errors, and the final evaluations are not distinguishable by a rank-sum test
    g = r["gpu_vs_cpu"]
    assert all(g["within_2se"]), g
    assert g["mannwhitney_p_final"] > 0.05
