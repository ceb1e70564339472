"""GPU parity at the headline size: 65,536 envs, the instantiations the bench and config 5 time.

Above 32,768 envs quad_step launches k_step_h with 256-env blocks (HB = 256: 512-thread blocks,
LDS images H[f*HB+l] / CT[...], the obs-row transpose and the helper waves' reset rows all sized
by HB), and the one-launch rollout runs k_rollout<..., SPEC=true> on reference-default handles.
The rest of the suite pins these forms at <= 5,000 envs, i.e. the 64-env blocks; here every row
of a full 65,536-env batch is checked against the float64 oracle (oracle/quad_oracle.c through
its batch entry points) under the suite's bar (tests/test_gpu_parity.py):

  * hover / trajectory x RateControlWrapper off / on, SPEC constants on / off;
  * the batch = the reference golden fixtures' pre-states and actions (golden_*_steps.npz, made by
    tools/gen_golden.py from the reference's own envs) tiled over the first rows, then random
    states (wide rates, every 16th env one step before its time limit, random episode counters);
  * auto_reset off: every row's obs, reward, flags, step counter, voltage, qpos / qvel, rate
    integral, motor commands, info["state"] vs the oracle; golden rows also vs the fixture;
  * auto_reset on (SB3 VecEnv semantics): terminal_observation of every finished env vs the
    oracle, its reset obs bit-exact with the oracle's Philox draw of (seed, global id, episode),
    counters reset, every other row as above;
  * k_rollout SPEC=true (one rollout step of quad_rollout from the same states): the env step of
    the clipped sampled action vs the oracle, the next obs (or reset obs) and the state.

Reference semantics: envs/hover_env.py:159-198, envs/trajectory_follow_env.py:145-174,
envs/rate_wrapper.py:69-106, SB3 DummyVecEnv auto-reset (train.py:48).
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from test_gpu_parity import (NON_EULER, _random_states, euler_combination_ok, euler_ok, obs_euler_of_quat,
                             operand_only, parity_ok)

pytestmark = pytest.mark.gpu

N_FULL = 65536
VARIANTS = [("hover", None, O.ENV_HOVER, O.WRAP_NONE, "hover_steps"),
            ("hover", "RateControlWrapper", O.ENV_HOVER, O.WRAP_CTBR, "ctbr_steps"),
            ("trajectory", None, O.ENV_TRAJ, O.WRAP_NONE, "traj_steps"),
            ("trajectory", "RateControlWrapper", O.ENV_TRAJ, O.WRAP_CTBR, "traj_ctbr_steps")]
IDS = ["hover", "hover_ctbr", "traj", "traj_ctbr"]
SEED, BASE = 0xC0FFEE, 1 << 20


@pytest.fixture(params=["1", "0"])
def spec_mode(request, monkeypatch):
    monkeypatch.setenv("QUADENV_SPEC", request.param)
    monkeypatch.delenv("QUADENV_HBLOCK", raising=False)
    monkeypatch.delenv("QUADENV_NT", raising=False)
    return request.param


def _batch(golden_dir, fixture, kind, wrap, n=N_FULL):
    """Golden pre-states + actions in the first rows, random states after (see module doc)."""
    d = np.load(os.path.join(golden_dir, f"golden_{fixture}.npz"))
    rng = np.random.default_rng(1000 + 10 * kind + wrap)
    st = _random_states(n, rng)
    acts = rng.uniform(-1.2, 1.2, (n, 4)).astype(np.float32)
    ng = len(d["action"])
    for f, k in (("qpos", "pre_qpos"), ("qvel", "pre_qvel"), ("voltage", "pre_voltage"),
                 ("target", "pre_target"), ("step_count", "pre_step"), ("rate_int", "pre_rate_int")):
        st[f][:ng] = d[k].astype(st[f].dtype)
    acts[:ng] = d["action"]
    limit = O.default_cfg(kind, wrap).max_episode_steps
    st["step_count"][ng::16] = limit - 1  # time-limit truncations among the random rows
    st["episode"] = rng.integers(0, 1 << 20, n).astype(np.uint32)
    return st, acts, d, ng


def _env(env_name, wrapper, auto_reset):
    from uav_reinforcement_learning_control_amd import _native as N
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    env = QuadVecEnv(N_FULL, env=env_name, wrapper=wrapper, device="cuda:0", seed=SEED,
                     env_id_base=BASE, auto_reset=auto_reset)
    return env, N.lib().quad_kernel_form(env._h)


def _check_rows(g, ref, st, rows, what):
    """The suite's bar on `rows` (vectorized); returns the failing row indices (and prints, for
    each, the fields that fail with got / oracle / pre-step values)."""
    ok = np.ones(len(rows), bool)
    fails = {}

    def note(name, m):
        nonlocal ok
        ok &= m
        for j in np.nonzero(~m)[0][:8]:
            fails.setdefault(int(rows[j]), []).append(name)

    note("terminated", g["terminated"][rows] == ref["terminated"][rows])
    note("truncated", g["truncated"][rows] == ref["truncated"][rows])
    for k in what:
        if k in ("qpos", "qvel"):
            note(k, parity_ok(g[k][rows], ref[k][rows], st[k][rows]))
        elif k == "rate_int":
            note(k, parity_ok(g["rate_int"][rows], ref["rate_int"][rows], st["rate_int"][rows], atol=1e-9))
        elif k == "state12":
            pre = np.concatenate([st["qpos"][rows][:, :3], np.zeros((len(rows), 3), np.float32),
                                  st["qvel"][rows][:, :6]], 1)
            note(k, parity_ok(g["state12"][rows][:, NON_EULER], ref["state12"][rows][:, NON_EULER], pre[:, NON_EULER]))
            note("euler", euler_ok(g["state12"][rows], None, g["qpos"][rows], ref["qpos"][rows]))
            note("roll-yaw", euler_combination_ok(g["state12"][rows], ref["state12"][rows]))
        elif k == "obs":
            # (reset rows carry the reset obs in both and are compared bit-exactly elsewhere); the
            # Euler columns against the conversion of the kernel's own quaternion (test_gpu_parity)
            note(k, parity_ok(g["obs"][rows][:, NON_EULER], ref["obs"][rows][:, NON_EULER]))
            note("obs-euler", parity_ok(g["obs"][rows][:, 3:6], obs_euler_of_quat(g["qpos"][rows])))
            note("quat", parity_ok(g["qpos"][rows][:, 3:7], ref["qpos"][rows][:, 3:7]))
        else:
            gk, rk = g[k][rows], ref[k][rows]
            if gk.ndim == 1:
                gk, rk = gk[:, None], rk[:, None]
            note(k, parity_ok(gk, rk))
    for i, names in list(fails.items())[:8]:
        print(f"\nrow {i} fails {names}")
        for k in names:
            if k in g and k in ref:
                print(f"  {k}: got {np.asarray(g[k][i]).tolist()}\n  {'':{len(k)}}  ref {np.asarray(ref[k][i]).tolist()}")
        print(f"  pre qpos {st['qpos'][i].tolist()}\n  pre qvel {st['qvel'][i].tolist()}")
    return rows[~ok]


def _operand_slack(g, ref, st, rows):
    nq, oq = operand_only(g["qpos"][rows], ref["qpos"][rows], st["qpos"][rows])
    nv, ov = operand_only(g["qvel"][rows], ref["qvel"][rows], st["qvel"][rows])
    assert len(oq) == len(ov) == 0, (oq[:5], ov[:5])
    assert nq + nv <= 0.01 * len(rows), (nq, nv)
    return nq + nv


@pytest.mark.parametrize("env_name,wrapper,kind,wrap,fixture", VARIANTS, ids=IDS)
def test_full_batch_step_matches_oracle(golden_dir, env_name, wrapper, kind, wrap, fixture, spec_mode):
    st, acts, d, ng = _batch(golden_dir, fixture, kind, wrap)
    env, form = _env(env_name, wrapper, auto_reset=False)
    # k_step_h, 256-env blocks, nt state policy: the headline's instantiation
    assert form == (32 | 128 | 256 | (16 if spec_mode == "1" else 0)), form
    env.set_state(**st)
    obs, rew, te, tr, inf = env.step(torch.from_numpy(acts).cuda(), info="full")
    torch.cuda.synchronize()
    post = env.get_state()
    g = dict(obs=obs.cpu().numpy(), reward=rew.cpu().numpy(), terminated=te.cpu().numpy(),
             truncated=tr.cpu().numpy(), state12=inf["state"].cpu().numpy(),
             motor_commands=inf["motor_commands"].cpu().numpy(), voltage=post["voltage"],
             qpos=post["qpos"], qvel=post["qvel"], rate_int=post["rate_int"])
    ref = O.step_batch(O.default_cfg(kind, wrap), st, acts)
    rows = np.arange(N_FULL)
    bad = _check_rows(g, ref, st, rows, ("obs", "reward", "voltage", "motor_commands", "qpos", "qvel",
                                          "state12", "rate_int"))
    assert len(bad) == 0, (len(bad), bad[:8])
    assert np.array_equal(post["step_count"], st["step_count"] + 1)
    assert np.array_equal(post["episode"], st["episode"])  # no auto-reset: counters untouched
    # the golden rows also against the reference's own outputs
    gr = np.arange(ng)
    assert np.array_equal(g["terminated"][gr], d["terminated"]) and np.array_equal(g["truncated"][gr], d["truncated"])
    assert parity_ok(g["obs"][gr], d["obs"]).all() and parity_ok(g["reward"][gr, None], d["reward"][:, None]).all()
    slack = _operand_slack(g, ref, st, rows)
    nterm, ntrunc = int(g["terminated"].sum()), int(g["truncated"].sum())
    print(f"\n{env_name}/{wrapper} spec {spec_mode}: {N_FULL} rows, {ng} golden, terminated {nterm}, "
          f"truncated {ntrunc}, operand-relative-only components {slack}")
    assert nterm > 300 and ntrunc > 1000  # the case exercised both flags (measured 424 .. 1,500 terminations)
    env.close()


@pytest.mark.parametrize("env_name,wrapper,kind,wrap,fixture", VARIANTS, ids=IDS)
def test_full_batch_auto_reset_matches_oracle(golden_dir, env_name, wrapper, kind, wrap, fixture, spec_mode):
    st, acts, d, ng = _batch(golden_dir, fixture, kind, wrap)
    env, form = _env(env_name, wrapper, auto_reset=True)
    assert form & 128, form
    env.set_state(**st)
    obs, rew, te, tr, inf = env.step(torch.from_numpy(acts).cuda(), info="full")
    torch.cuda.synchronize()
    post = env.get_state()
    te, tr = te.cpu().numpy(), tr.cpu().numpy()
    g = dict(obs=obs.cpu().numpy(), reward=rew.cpu().numpy(), terminated=te, truncated=tr,
             term_obs=inf["terminal_observation"].cpu().numpy(),
             tl=inf["TimeLimit.truncated"].cpu().numpy(), qpos=post["qpos"], qvel=post["qvel"],
             rate_int=post["rate_int"], voltage=post["voltage"])
    cfg = O.default_cfg(kind, wrap)
    ref = O.step_batch(cfg, st, acts)
    done = te | tr
    dr, nr = np.nonzero(done)[0], np.nonzero(~done)[0]
    assert np.array_equal(g["tl"], tr & ~te)
    # envs that go on: the same bar as without auto-reset
    bad = _check_rows(g, ref, st, nr, ("obs", "reward", "voltage", "qpos", "qvel", "rate_int"))
    assert len(bad) == 0, (len(bad), bad[:8])
    assert np.array_equal(post["step_count"][nr], st["step_count"][nr] + 1)
    assert np.array_equal(post["episode"][nr], st["episode"][nr])
    # envs that finished: flags, reward and terminal observation of the step, then the reset
    assert np.array_equal(te[dr], ref["terminated"][dr]) and np.array_equal(tr[dr], ref["truncated"][dr])
    assert parity_ok(g["term_obs"][dr], ref["obs"][dr]).all()
    assert parity_ok(g["reward"][dr, None], ref["reward"][dr, None]).all()
    reset_obs = O.reset_obs_batch(cfg, SEED, BASE + dr.astype(np.uint64), st["episode"][dr])
    assert np.array_equal(g["obs"][dr].view(np.uint32), reset_obs.view(np.uint32)), \
        int(np.sum(np.any(g["obs"][dr] != reset_obs, axis=1)))
    assert np.all(post["step_count"][dr] == 0) and np.array_equal(post["episode"][dr], st["episode"][dr] + 1)
    i12, t3 = O.reset_draw_batch(cfg, SEED, BASE + dr.astype(np.uint64), st["episode"][dr])
    assert np.array_equal(post["qpos"][dr, :3], i12[:, :3]) and np.array_equal(post["qvel"][dr, :6], i12[:, 6:])
    assert np.all(post["qpos"][dr, 7:] == 0) and np.all(post["qvel"][dr, 6:] == 0)
    assert np.array_equal(post["target"][dr], i12[:, :3] if kind == O.ENV_TRAJ else t3)
    if wrap == O.WRAP_CTBR:
        assert np.all(post["rate_int"][dr] == 0)
    print(f"\n{env_name}/{wrapper} spec {spec_mode}: {len(dr)} auto-resets of {N_FULL}")
    assert len(dr) > 2000
    env.close()


@pytest.mark.parametrize("env_name,wrapper,kind,wrap,fixture", VARIANTS, ids=IDS)
def test_full_batch_rollout_first_step_matches_oracle(golden_dir, env_name, wrapper, kind, wrap, fixture,
                                                       spec_mode):
    """quad_rollout (k_rollout<KIND, CTBR, 2, SPEC>) for one step from the batch: the sampled action,
    clipped to the action space, is what the env steps (the oracle from the same state), the
    next obs row is the stepped obs or the bit-exact reset obs, the reward row is the step's
    reward (plus the critic bootstrap on a time-limit truncation, not re-checked here), and the
    carried env state is the oracle's."""
    from test_gpu_rollout import _bufs, _policy
    from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy
    st, _, d, ng = _batch(golden_dir, fixture, kind, wrap)
    env, form = _env(env_name, wrapper, auto_reset=True)
    env.set_state(**st)
    pol = _policy()
    with torch.no_grad():  # a wide action distribution: some samples leave [-1, 1] and are clipped
        pol.log_std.fill_(-0.2)
    fp = FusedPolicy(pol)
    fp.pack()
    b = _bufs(1, N_FULL)
    env.observe(out=b["last_obs"])
    obs0 = b["last_obs"].clone()
    b["last_start"].zero_()
    fp.rollout(env, t0=0, steps=1, seed=0x5EED, gamma=0.99, **b)
    torch.cuda.synchronize()
    post = env.get_state()
    acts = b["actions"][0].cpu().numpy()
    assert np.isfinite(acts).all() and (np.abs(acts) > 1).any()  # the clip is exercised
    cfg = O.default_cfg(kind, wrap)
    ref = O.step_batch(cfg, st, np.clip(acts, -1, 1))
    nxt = b["last_obs"].cpu().numpy()
    starts = b["last_start"].cpu().numpy()
    rew = b["rewards"][0].cpu().numpy()
    done = ref["terminated"] | ref["truncated"]
    assert np.array_equal(starts == 1, done)
    dr, nr = np.nonzero(done)[0], np.nonzero(~done)[0]
    g = dict(obs=nxt, reward=rew, terminated=ref["terminated"], truncated=ref["truncated"],
             qpos=post["qpos"], qvel=post["qvel"], rate_int=post["rate_int"], voltage=post["voltage"])
    bad = _check_rows(g, ref, st, nr, ("obs", "reward", "voltage", "qpos", "qvel", "rate_int"))
    assert len(bad) == 0, (len(bad), bad[:8])
    term = np.nonzero(ref["terminated"])[0]
    assert parity_ok(rew[term, None], ref["reward"][term, None]).all()
    reset_obs = O.reset_obs_batch(cfg, SEED, BASE + dr.astype(np.uint64), st["episode"][dr])
    assert np.array_equal(nxt[dr].view(np.uint32), reset_obs.view(np.uint32))
    assert np.all(post["step_count"][dr] == 0) and np.array_equal(post["episode"][dr], st["episode"][dr] + 1)
    assert np.array_equal(post["step_count"][nr], st["step_count"][nr] + 1)
    assert torch.equal(b["obs_copy"][0], obs0)  # the buffer's obs row is the observation the policy saw
    print(f"\nrollout {env_name}/{wrapper} spec {spec_mode}: {len(dr)} resets, {len(nr)} stepped rows")
    env.close()
