"""Batched evaluation: the waypoint bookkeeping kernel and the batched
drivers against a CPU restatement of evaluate.py's per-env loop (oracle env + torch policy).

Tolerances: positions / rewards of the GPU run vs the CPU loop within 1e-4 (the MFMA policy and
the float32 env differ from torch-CPU + float64 oracle by ~1e-6 per step); step counts, waypoint
counters and statuses exactly.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _policy(seed=0):
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    torch.manual_seed(seed)
    return ActorCritic()


def test_waypoint_switching_and_lap_with_large_radius():
    """reach_radius larger than the course: every step reaches the current waypoint, so a lap of
    n waypoints ends after n - 1 steps (evaluate.py starts at WP #0 targeting WP #1)."""
    from uav_reinforcement_learning_control_amd.evaluate import evaluate_waypoints
    pol = _policy()
    with torch.no_grad():  # ~hover thrust: (a + 1) / 2 * 52 N ~ m g
        pol.action_net.bias.copy_(torch.tensor([-0.915, 0.0, 0.0, 0.0]))
    r = evaluate_waypoints(pol, ["eight", "circle", "square"], [0.5, 0.8], reach_radius=50.0,
                           max_steps=200)
    assert np.all(r["status"] == 1) and np.all(r["laps"] == 1)
    assert np.array_equal(r["steps"], r["n_waypoints"] - 1)
    assert np.array_equal(r["reached"], r["n_waypoints"] - 1)
    assert np.array_equal(r["wp_idx"], np.zeros_like(r["wp_idx"]))


def _cpu_waypoint_loop(policy, wps, reach, max_steps, wrapper=O.WRAP_NONE):
    """evaluate.py:440-612 restated on the CPU oracle (no viewer)."""
    cfg = O.default_cfg(O.ENV_HOVER, wrapper)
    cfg.max_episode_steps = max_steps
    e = O.Env(cfg=cfg)
    k = 1 % len(wps)
    e.set_full_state(np.r_[wps[0], [1, 0, 0, 0], [0, 0, 0, 0]], np.zeros(10), 8.4,
                     wps[k].astype(np.float32), 0)
    obs = np.zeros(12, np.float32)
    O.lib().oracle_get_obs(C.byref(cfg), C.byref(e.s), O._fp(obs))
    total, steps, reached, laps, status, pos = 0.0, 0, 0, 0, 0, []
    while status == 0:
        with torch.no_grad():
            mean, _ = policy.forward_heads(torch.from_numpy(obs[None]))
        a = np.clip(mean[0].numpy(), -1, 1).astype(np.float32)
        out = O.out_to_dict(e.step(a))
        obs = out["obs"]
        total += out["reward"]
        steps += 1
        p = out["state12"][:3]
        pos.append(p)
        if float(np.linalg.norm(p - wps[k])) < reach:
            reached += 1
            k = (k + 1) % len(wps)
            if k == 0:
                laps += 1
                status = 1
            else:
                e.s.target[:] = [float(x) for x in wps[k].astype(np.float32)]
        if status == 0 and out["terminated"]:
            status = 2
        elif status == 0 and out["truncated"]:
            status = 3
    return dict(total=total, steps=steps, reached=reached, laps=laps, status=status, pos=np.array(pos))


@pytest.mark.parametrize("reach", [0.25, 0.6])
def test_waypoint_eval_matches_cpu_loop(reach):
    from uav_reinforcement_learning_control_amd.evaluate import evaluate_waypoints
    from uav_reinforcement_learning_control_amd.utils.trajectories import make_trajectory
    pol = _policy(3)
    with torch.no_grad():  # a policy that moves: non-trivial head
        pol.action_net.weight.mul_(60.0)
        pol.action_net.bias.copy_(torch.tensor([-0.83, 0.0, 0.0, 0.0]))
    names = ["eight", "circle", "square"]
    r = evaluate_waypoints(pol, names, [0.5], reach_radius=reach, max_steps=400, record=True)
    for i, nm in enumerate(names):
        ref = _cpu_waypoint_loop(pol, make_trajectory(nm, spacing=0.5), reach, 400)
        assert (r["status"][i], r["steps"][i], r["reached"][i], r["laps"][i]) == \
            (ref["status"], ref["steps"], ref["reached"], ref["laps"]), (nm, ref["status"], ref["steps"])
        assert abs(r["total_reward"][i] - ref["total"]) <= 1e-4 * max(1.0, abs(ref["total"]))
        np.testing.assert_allclose(r["positions"][:ref["steps"], i], ref["pos"], atol=1e-4)


def test_episode_eval_properties_and_determinism():
    from uav_reinforcement_learning_control_amd.evaluate import evaluate_episodes
    pol = _policy(5)
    a = evaluate_episodes(pol, num_episodes=2048, max_episode_steps=300, seed=4)
    b = evaluate_episodes(pol, num_episodes=2048, max_episode_steps=300, seed=4)
    assert np.array_equal(a["rewards"], b["rewards"]) and np.array_equal(a["lengths"], b["lengths"])
    assert np.all((a["lengths"] >= 1) & (a["lengths"] <= 300))
    assert np.all(a["rewards"] >= 0) and np.all(a["rewards"] <= a["lengths"] + 1e-9)
    assert np.all(a["terminated"] | (a["lengths"] == 300))
