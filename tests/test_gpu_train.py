"""The training driver's reference callbacks (train.py:71-86: CheckpointCallback, EvalCallback with
best-model save) and resume; the wrapper facades' reference attributes (rate_wrapper.py:26-111,
wrappers.py:13-36) on the GPU env."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_train_checkpoints_eval_and_resume(tmp_path):
    from uav_reinforcement_learning_control_amd import train
    from uav_reinforcement_learning_control_amd.export import load_sb3_policy
    args = ["--num-envs", "1024", "--n-steps", "16", "--n-epochs", "1", "--n-minibatches", "4",
            "--total-timesteps", str(3 * 1024 * 16), "--checkpoint-freq", str(2 * 1024 * 16),
            "--eval-freq", str(1024 * 16), "--n-eval-episodes", "8",
            "--log-dir", str(tmp_path / "logs"), "--model-dir", str(tmp_path / "models")]
    train.main(args)
    (mdir,) = glob.glob(str(tmp_path / "models" / "*"))
    (ldir,) = glob.glob(str(tmp_path / "logs" / "*"))
    ck = sorted(glob.glob(os.path.join(mdir, "hover_policy_*_steps.zip")))
    assert [os.path.basename(p) for p in ck] == [f"hover_policy_{2 * 1024 * 16}_steps.zip"]
    assert os.path.exists(ck[0][:-4] + ".pt")
    assert os.path.exists(os.path.join(mdir, "best_model.zip"))
    assert os.path.exists(os.path.join(mdir, "hover_policy_final.zip"))
    ev = np.load(os.path.join(ldir, "evaluations.npz"))
    assert list(ev["timesteps"]) == [1024 * 16 * k for k in (1, 2, 3)]
    assert ev["results"].shape == (3, 8) and ev["ep_lengths"].shape == (3, 8)
    best = load_sb3_policy(os.path.join(mdir, "best_model.zip"))
    assert best is not None
    # resume from the step-32768 checkpoint: timesteps continue, parameters start where they were
    sd = torch.load(ck[0][:-4] + ".pt", map_location="cpu", weights_only=True)
    assert sd["num_timesteps"] == 2 * 1024 * 16 and sd["noise_step"] == 2 * 16
    args2 = [a if a != str(3 * 1024 * 16) else str(4 * 1024 * 16) for a in args]
    args2 = [x for x in args2] + ["--resume", ck[0][:-4] + ".pt"]
    args2[args2.index(str(tmp_path / "models"))] = str(tmp_path / "models2")
    args2[args2.index(str(tmp_path / "logs"))] = str(tmp_path / "logs2")
    train.main(args2)
    (ldir2,) = glob.glob(str(tmp_path / "logs2" / "*"))
    rows = open(os.path.join(ldir2, "progress.csv")).read().strip().splitlines()[1:]
    assert [int(r.split(",")[1]) for r in rows] == [3 * 1024 * 16, 4 * 1024 * 16]


def test_rate_wrapper_facade_exposes_reference_state():
    from uav_reinforcement_learning_control_amd.envs import HoverEnv, QuadVecEnv, RateControlWrapper, get_wrapper
    env = RateControlWrapper(HoverEnv(device="cuda:0"))
    assert isinstance(env, RateControlWrapper) and get_wrapper("RateControlWrapper") is RateControlWrapper
    assert isinstance(env.unwrapped, HoverEnv)
    np.testing.assert_allclose(env.kd, [26, 26, 18]) and np.testing.assert_allclose(env.inertia, [4.16e-4, 4.23e-4, 5.37e-4])
    assert env.ki_rate_torque == 0.025 and env.integral_max == 0.01 and env._dt == 0.01
    assert abs(env.max_rate_rad - np.deg2rad(360.0)) < 1e-12
    obs, info = env.reset(seed=3)
    assert np.array_equal(env._rate_int_torque, np.zeros(3))
    a = np.array([0.1, 0.3, -0.2, 0.05], np.float32)
    s12 = info["state"]
    obs, r, te, tr, info = env.step(a)
    # the integral after one step: clip(ki dt (des - w), +-imax) (rate_wrapper.py:84-88) in float64
    des = a[1:].astype(np.float64) * np.deg2rad(360.0)
    ref = np.clip(0.025 * 0.01 * (des - s12[9:12].astype(np.float64)), -0.01, 0.01)
    np.testing.assert_allclose(env._rate_int_torque, ref, rtol=1e-6, atol=1e-9)
    assert np.array_equal(env.unwrapped._prev_action, a)   # rate_wrapper.py:105
    env._rate_int_torque = np.array([0.001, -0.002, 0.003])
    np.testing.assert_allclose(env._rate_int_torque, [0.001, -0.002, 0.003], rtol=1e-6)
    env.close()
    # vectorized: the facade steps the CTBR kernel (bit-identical to building it directly)
    n = 256
    w = RateControlWrapper(QuadVecEnv(n, device="cuda:0", seed=4))
    d = QuadVecEnv(n, wrapper="RateControlWrapper", device="cuda:0", seed=4)
    assert torch.equal(w.reset(), d.reset())
    for k in range(5):
        acts = d.random_actions(k)
        o1 = w.step(acts)[0].clone()
        o2 = d.step(acts)[0]
        assert torch.equal(o1, o2)
    assert w._rate_int_torque.shape == (n, 3) and w.num_envs == n
    w.close(); d.close()


def test_relpos_wrapper_facade():
    from uav_reinforcement_learning_control_amd.envs import HoverEnv, get_wrapper
    env = get_wrapper("RelPosActWrapper")(HoverEnv(device="cuda:0"))
    obs, _ = env.reset(seed=1)
    assert obs.shape == (7,) and np.all(obs[3:] == 0)
    a = np.array([0.2, -0.1, 0.3, 0.0], np.float32)
    obs, *_ = env.step(a)
    assert np.array_equal(obs[3:], a) and np.array_equal(env.observation(np.arange(12, dtype=np.float32))[3:], a)
    assert env.observation_space.shape == (7,)
    env.close()


def test_relpos_over_rate_control_stack():
    """The README's stack RelPosActWrapper(RateControlWrapper(HoverEnv())): the CTBR controller stays
    in the step (combined kernel kind QUAD_WRAP_CTBR_RELPOS) and obs7 carries the rate action
    (rate_wrapper.py:100-106); bit-identical to building that kind directly; wrapping keeps the
    wrapped env's seed and cfg overrides; the reverse order is refused with an explanation."""
    from uav_reinforcement_learning_control_amd import _native as N
    from uav_reinforcement_learning_control_amd.envs import (HoverEnv, QuadVecEnv, RateControlWrapper,
                                                             RelPosActWrapper)
    env = RelPosActWrapper(RateControlWrapper(HoverEnv(device="cuda:0", seed=7, density=0.9), kd=[20, 20, 10]))
    assert isinstance(env.env, RateControlWrapper) and env.observation_space.shape == (7,)
    cfg = env.unwrapped._vec.cfg
    assert cfg.wrapper == N.WRAP_CTBR_RELPOS and abs(cfg.density - 0.9) < 1e-12
    np.testing.assert_allclose(cfg.rate_kd[:], [20, 20, 10])
    assert env.unwrapped._vec.seed_value == 7
    obs, _ = env.reset(seed=2)
    assert obs.shape == (7,) and np.all(obs[3:] == 0)
    a = np.array([0.1, 0.4, -0.3, 0.2], np.float32)
    obs, *_ = env.step(a)
    assert np.array_equal(obs[3:], a)                         # the RATE action, not the torques
    assert np.any(env.env._rate_int_torque != 0)              # the controller ran
    env.close()
    # vectorized: the facade stack steps exactly the combined kind
    n = 512
    w = RelPosActWrapper(RateControlWrapper(QuadVecEnv(n, device="cuda:0", seed=4)))
    d = QuadVecEnv(n, wrapper="ctbr_relpos", device="cuda:0", seed=4)
    assert torch.equal(w.reset(), d.reset())
    for k in range(6):
        acts = d.random_actions(k)
        o1 = w.step(acts)[0].clone()
        o2, _, te, tr, _ = d.step(acts)
        live = ~(te | tr)  # (auto-reset rows carry the reset obs: previous action zeros)
        assert torch.equal(o1, o2) and torch.equal(o2[live][:, 3:], acts[live])
    w.close(); d.close()
    with pytest.raises(TypeError):
        RateControlWrapper(RelPosActWrapper(HoverEnv(device="cuda:0")))
    # the intermediate RateControlWrapper now passes obs7 up: its space says so
    w = RelPosActWrapper(RateControlWrapper(QuadVecEnv(64, device="cuda:0", seed=4)))
    assert w.env.observation_space.shape == (7,) and w.observation_space.shape == (7,)
    w.close()
    # envs BUILT with the CTBR kind keep the rate controller under RelPosActWrapper (no silent
    # downgrade to raw torques); an observation wrapper twice is refused
    for base in (QuadVecEnv(64, wrapper="ctbr", device="cuda:0", seed=4),
                 HoverEnv(device="cuda:0", wrapper="RateControlWrapper")):
        w = RelPosActWrapper(base)
        vec = w.env if isinstance(w.env, QuadVecEnv) else w.unwrapped._vec
        assert vec.cfg.wrapper == N.WRAP_CTBR_RELPOS
        with pytest.raises(TypeError):
            RelPosActWrapper(w.env)
        w.close()


@pytest.mark.parametrize("one_launch", [True, False])
def test_resume_draws_fresh_noise(one_launch):
    """PPO.state_dict / load_state_dict (train.py --resume): a resumed run's rollouts draw the
    action noise that follows the checkpoint, not the original run's from step 0 -- on the one-launch
    path (quad_rollout, keyed by the host step counter) and the two-launch path (policy kernel +
    env step, keyed by the device cursor, which graph capture zeroes)."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPO, PPOConfig
    cfg = PPOConfig(n_steps=16, n_minibatches=2, n_epochs=1, fused_rollout=one_launch)

    def run(sd=None, rollouts=1):
        env = QuadVecEnv(512, env="hover", device="cuda:0", seed=9)
        algo = PPO(env, cfg, seed=2)
        assert algo._one_launch == one_launch
        if sd is not None:
            algo.load_state_dict(sd)
        acts = []
        for _ in range(rollouts):
            algo.collect_rollouts()
            acts.append(algo.buf_act.clone())
        out = algo.state_dict(), acts
        env.close()
        return out

    sd, (a_first, a_second) = run(rollouts=2)
    assert sd["noise_step"] == 2 * 16
    sd_b, (b_first,) = run(sd)  # same params, same env seed: only the noise can differ
    assert not torch.equal(b_first, a_first)  # not a replay of the original run's first rollout
    # where the counter resumed: the rollout after the checkpoint consumed noise steps 32 .. 47
    assert sd_b["noise_step"] == 2 * 16 + 16
    # a checkpoint between rollout boundaries: the one-launch path continues at the saved step, the
    # two-launch path (whose cursor also selects the buffer row t % n_steps) at the next boundary
    sd_mid = dict(sd, noise_step=20)
    sd_c, _ = run(sd_mid)
    assert sd_c["noise_step"] == (20 + 16 if one_launch else 32 + 16)
