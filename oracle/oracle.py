"""ctypes binding of the CPU float64 oracle -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker (never as the measured or shipped path).  The library is
built from ``oracle/quad_oracle.c`` by ``oracle/Makefile`` (``build()`` in ``__graft_entry__``).

See ``oracle/quad_oracle.h`` for what each entry point restates (reference file:line) and the
pinning status (env semantics pinned by golden vectors; MuJoCo physics "parity unpinned").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libquadoracle.so")

ENV_HOVER, ENV_TRAJ, ENV_BRAX_HOVER, ENV_BRAX_TRAJ = 0, 1, 2, 3
WRAP_NONE, WRAP_CTBR, WRAP_RELPOS, WRAP_CTBR_RELPOS = 0, 1, 2, 3


class OracleOpt(C.Structure):
    _fields_ = [("timestep", C.c_double), ("gravity", C.c_double * 3),
                ("density", C.c_double), ("viscosity", C.c_double)]


class OracleCfg(C.Structure):
    _fields_ = [
        ("env_kind", C.c_int32), ("wrapper", C.c_int32), ("max_episode_steps", C.c_int32),
        ("pad_", C.c_int32),
        ("obs_low", C.c_float * 12), ("obs_high", C.c_float * 12),
        ("init_low", C.c_float * 12), ("init_high", C.c_float * 12),
        ("target_low", C.c_float * 3), ("target_high", C.c_float * 3),
        ("term_low", C.c_float * 12), ("term_high", C.c_float * 12),
        ("act_low", C.c_float * 4), ("act_high", C.c_float * 4),
        ("max_motor_thrust", C.c_double), ("arm_length", C.c_double), ("yaw_coeff", C.c_double),
        ("nominal_voltage", C.c_double), ("min_voltage", C.c_double),
        ("vdrop_base", C.c_double), ("vdrop_load", C.c_double),
        ("rate_max_rad", C.c_double), ("rate_kd", C.c_double * 3), ("rate_ki", C.c_double),
        ("rate_imax", C.c_double), ("inertia", C.c_double * 3), ("max_torque", C.c_double),
        ("opt", OracleOpt),
    ]


class OracleEnv(C.Structure):
    _fields_ = [("qpos", C.c_double * 11), ("qvel", C.c_double * 10), ("voltage", C.c_double),
                ("target", C.c_float * 3), ("step_count", C.c_int32),
                ("rate_int", C.c_double * 3), ("state12", C.c_float * 12),
                ("prev_action", C.c_float * 4)]


class OracleStepOut(C.Structure):
    _fields_ = [("obs", C.c_float * 12), ("reward", C.c_double), ("terminated", C.c_int32),
                ("truncated", C.c_int32), ("state12", C.c_float * 12),
                ("motor_commands", C.c_double * 4), ("voltage", C.c_double),
                ("voltage_scale", C.c_double), ("env_action", C.c_float * 4), ("obs7", C.c_float * 7)]


class OracleBraxCfg(C.Structure):
    _fields_ = [("kind", C.c_int32), ("episode_length", C.c_int32), ("target", C.c_float * 3),
                ("pos_limit_xy", C.c_float), ("pos_limit_z_low", C.c_float),
                ("pos_limit_z_high", C.c_float), ("vel_limit", C.c_float),
                ("reset_noise", C.c_float), ("reward_pos_coef", C.c_float),
                ("reward_action_coef", C.c_float), ("ctrl_min", C.c_float * 4),
                ("ctrl_max", C.c_float * 4), ("traj_center", C.c_float * 3),
                ("traj_amp", C.c_float * 3), ("traj_freq", C.c_float * 3),
                ("traj_duration", C.c_float), ("max_motor_thrust", C.c_double),
                ("arm_length", C.c_double), ("yaw_coeff", C.c_double), ("opt", OracleOpt)]


class OracleBraxEnv(C.Structure):
    _fields_ = [("qpos", C.c_double * 11), ("qvel", C.c_double * 10),
                ("first_qpos", C.c_double * 11), ("first_qvel", C.c_double * 10),
                ("steps", C.c_int32), ("env_steps", C.c_int32)]


class OracleBraxOut(C.Structure):
    _fields_ = [("obs", C.c_float * 21), ("terminal_obs", C.c_float * 21), ("reward", C.c_double),
                ("terminated", C.c_int32), ("truncated", C.c_int32),
                ("motor_commands", C.c_double * 4), ("target", C.c_float * 3)]


_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        dp = C.POINTER(C.c_double)
        fp = C.POINTER(C.c_float)
        L.oracle_default_cfg.argtypes = [C.c_int32, C.c_int32, C.POINTER(OracleCfg)]
        L.oracle_mj_step.argtypes = [C.POINTER(OracleOpt), dp, dp, dp]
        L.oracle_mj_step.restype = C.c_int
        L.oracle_mj_forward.argtypes = [C.POINTER(OracleOpt), dp, dp, dp, dp, dp, dp, dp, dp]
        L.oracle_quat_to_euler.argtypes = [dp, dp]
        L.oracle_euler_to_quat.argtypes = [dp, dp]
        L.oracle_quat_to_euler_batch.argtypes = [dp, C.c_int32, dp]
        L.oracle_get_obs.argtypes = [C.POINTER(OracleCfg), C.POINTER(OracleEnv), fp]
        L.oracle_relpos_obs.argtypes = [C.POINTER(OracleEnv), fp, fp]
        L.oracle_env_reset.argtypes = [C.POINTER(OracleCfg), C.POINTER(OracleEnv), fp, fp, fp]
        L.oracle_env_step.argtypes = [C.POINTER(OracleCfg), C.POINTER(OracleEnv), fp,
                                      C.POINTER(OracleStepOut)]
        L.oracle_env_step_batch.argtypes = [C.POINTER(OracleCfg), C.POINTER(OracleEnv), C.c_int32,
                                            fp, C.POINTER(OracleStepOut)]
        L.oracle_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                           C.POINTER(C.c_uint32)]
        L.oracle_reset_draw.argtypes = [C.POINTER(OracleCfg), C.c_uint64, C.c_uint64, C.c_uint32,
                                        fp, fp]
        L.oracle_reset_draw_batch.argtypes = [C.POINTER(OracleCfg), C.c_uint64, C.c_void_p, C.c_void_p,
                                              C.c_int32, fp, fp]
        L.oracle_env_reset_batch.argtypes = [C.POINTER(OracleCfg), C.POINTER(OracleEnv), C.c_int32, fp, fp, fp]
        L.oracle_env_prepare_batch.argtypes = [C.POINTER(OracleCfg), C.POINTER(OracleEnv), C.c_int32]
        L.oracle_random_action.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, fp]
        L.oracle_bench_rollout.argtypes = [C.POINTER(OracleCfg), C.c_int32, C.c_int32, C.c_uint64]
        L.oracle_bench_rollout.restype = C.c_double
        L.oracle_mjx_step.argtypes = [C.POINTER(OracleOpt), dp, dp, dp]
        L.oracle_brax_default_cfg.argtypes = [C.c_int32, C.POINTER(OracleBraxCfg)]
        L.oracle_brax_reset_draw.argtypes = [C.POINTER(OracleBraxCfg), C.c_uint64, C.c_uint64,
                                             C.c_uint32, fp]
        L.oracle_brax_reset.argtypes = [C.POINTER(OracleBraxCfg), C.POINTER(OracleBraxEnv), fp, fp]
        L.oracle_brax_step.argtypes = [C.POINTER(OracleBraxCfg), C.POINTER(OracleBraxEnv), fp,
                                       C.c_int32, C.POINTER(OracleBraxOut)]
        for n in ("oracle_sizeof_env", "oracle_sizeof_stepout", "oracle_sizeof_cfg",
                  "oracle_sizeof_brax_cfg", "oracle_sizeof_brax_env", "oracle_sizeof_brax_out"):
            getattr(L, n).restype = C.c_size_t
        assert L.oracle_sizeof_brax_cfg() == C.sizeof(OracleBraxCfg)
        assert L.oracle_sizeof_brax_env() == C.sizeof(OracleBraxEnv)
        assert L.oracle_sizeof_brax_out() == C.sizeof(OracleBraxOut)
        assert L.oracle_sizeof_env() == C.sizeof(OracleEnv)
        assert L.oracle_sizeof_stepout() == C.sizeof(OracleStepOut)
        assert L.oracle_sizeof_cfg() == C.sizeof(OracleCfg)
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def default_cfg(env_kind: int = ENV_HOVER, wrapper: int = WRAP_NONE) -> OracleCfg:
    c = OracleCfg()
    lib().oracle_default_cfg(env_kind, wrapper, C.byref(c))
    return c


def default_opt() -> OracleOpt:
    return default_cfg().opt


def mj_step(qpos, qvel, ctrl, opt: OracleOpt | None = None):
    """mujoco.mj_step restated; returns (qpos', qvel', ctrl', warning_mask)."""
    opt = opt or default_opt()
    qp = np.array(qpos, dtype=np.float64).copy()
    qv = np.array(qvel, dtype=np.float64).copy()
    ct = np.array(ctrl, dtype=np.float64).copy()
    w = lib().oracle_mj_step(C.byref(opt), _dp(qp), _dp(qv), _dp(ct))
    return qp, qv, ct, w


def mj_forward(qpos, qvel, ctrl, opt: OracleOpt | None = None):
    opt = opt or default_opt()
    qp = np.ascontiguousarray(qpos, dtype=np.float64)
    qv = np.ascontiguousarray(qvel, dtype=np.float64)
    ct = np.ascontiguousarray(ctrl, dtype=np.float64)
    M = np.zeros((10, 10)); bias = np.zeros(10); pas = np.zeros(10); act = np.zeros(10)
    qacc = np.zeros(10)
    lib().oracle_mj_forward(C.byref(opt), _dp(qp), _dp(qv), _dp(ct), _dp(M), _dp(bias),
                            _dp(pas), _dp(act), _dp(qacc))
    return dict(M=M, bias=bias, passive=pas, actuator=act, qacc=qacc)


def quat_to_euler(q_wxyz):
    q = np.ascontiguousarray(q_wxyz, dtype=np.float64)
    e = np.zeros(3)
    lib().oracle_quat_to_euler(_dp(q), _dp(e))
    return e


def quat_to_euler_batch(q_wxyz):
    """[n, 4] wxyz quaternions -> [n, 3] float64 scipy as_euler('xyz') angles (oracle_quat_to_euler)."""
    q = np.ascontiguousarray(np.asarray(q_wxyz, np.float64).reshape(-1, 4))
    e = np.zeros((q.shape[0], 3))
    lib().oracle_quat_to_euler_batch(_dp(q), q.shape[0], _dp(e))
    return e


def euler_to_quat(e):
    ee = np.ascontiguousarray(e, dtype=np.float64)
    q = np.zeros(4)
    lib().oracle_euler_to_quat(_dp(ee), _dp(q))
    return q


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def reset_draw(cfg: OracleCfg, seed: int, gid: int, episode: int):
    i12 = np.zeros(12, np.float32)
    t3 = np.zeros(3, np.float32)
    lib().oracle_reset_draw(C.byref(cfg), seed, gid, episode, _fp(i12), _fp(t3))
    return i12, t3


def reset_draw_batch(cfg: OracleCfg, seed: int, gids, episodes):
    """reset_draw for many (global env id, episode) pairs: (init12 [n,12], target3 [n,3])."""
    g = np.ascontiguousarray(gids, np.uint64)
    e = np.ascontiguousarray(episodes, np.uint32)
    n = len(g)
    i12 = np.zeros((n, 12), np.float32)
    t3 = np.zeros((n, 3), np.float32)
    lib().oracle_reset_draw_batch(C.byref(cfg), seed, g.ctypes.data, e.ctypes.data, n, _fp(i12), _fp(t3))
    return i12, t3


def reset_obs_batch(cfg: OracleCfg, seed: int, gids, episodes):
    """The reset observation of each (global env id, episode) draw: Env.reset_with(reset_draw(...))."""
    i12, t3 = reset_draw_batch(cfg, seed, gids, episodes)
    n = len(i12)
    envs = (OracleEnv * n)()
    obs = np.zeros((n, 12), np.float32)
    lib().oracle_env_reset_batch(C.byref(cfg), envs, n, _fp(i12), _fp(t3), _fp(obs))
    return obs


def _as_struct_array(arr, ctype):
    import warnings
    with warnings.catch_warnings():  # ctypes' PEP 3118 format of a padded struct: numpy guesses right
        warnings.simplefilter("ignore", RuntimeWarning)
        v = np.ctypeslib.as_array(arr)
    assert v.dtype.itemsize == C.sizeof(ctype)
    return v


def step_batch(cfg: OracleCfg, st: dict, acts) -> dict:
    """One oracle step of many envs from the given float32 states (the dict of QuadVecEnv.get_state:
    qpos [n,11], qvel [n,10], voltage [n], target [n,3], step_count [n], rate_int [n,3],
    optionally prev_action [n,4]) -- Env.set_full_state + Env.step per row, in C. Returns the step
    outputs (obs, reward, terminated, truncated, state12, motor_commands, voltage, voltage_scale,
    env_action, obs7) and the post-step qpos / qvel / rate_int, as arrays over the rows."""
    a = np.ascontiguousarray(acts, np.float32)
    n = len(a)
    envs = (OracleEnv * n)()
    v = _as_struct_array(envs, OracleEnv)
    v["qpos"] = np.asarray(st["qpos"], np.float32)
    v["qvel"] = np.asarray(st["qvel"], np.float32)
    v["voltage"] = np.asarray(st["voltage"], np.float32)
    v["target"] = np.asarray(st["target"], np.float32)
    v["step_count"] = np.asarray(st["step_count"], np.int32)
    v["rate_int"] = np.asarray(st.get("rate_int", np.zeros((n, 3))), np.float32)
    v["prev_action"] = np.asarray(st.get("prev_action", np.zeros((n, 4))), np.float32)
    L = lib()
    L.oracle_env_prepare_batch(C.byref(cfg), envs, n)
    outs = (OracleStepOut * n)()
    L.oracle_env_step_batch(C.byref(cfg), envs, n, _fp(a), outs)
    o = _as_struct_array(outs, OracleStepOut)
    res = {k: np.array(o[k]) for k in o.dtype.names}
    res["terminated"] = res["terminated"].astype(bool)
    res["truncated"] = res["truncated"].astype(bool)
    res.update(qpos=np.array(v["qpos"]), qvel=np.array(v["qvel"]), rate_int=np.array(v["rate_int"]),
               step_count=np.array(v["step_count"]))
    return res


def random_action(seed: int, gid: int, step: int):
    a = np.zeros(4, np.float32)
    lib().oracle_random_action(seed, gid, step, _fp(a))
    return a


def bench_rollout(n_envs: int, n_steps: int, seed: int = 0, env_kind: int = ENV_HOVER,
                  wrapper: int = WRAP_NONE) -> float:
    cfg = default_cfg(env_kind, wrapper)
    return lib().oracle_bench_rollout(C.byref(cfg), n_envs, n_steps, seed)


class Env:
    """One reference env (HoverEnv / TrajectoryFollowEnv, optionally CTBR-wrapped)."""

    def __init__(self, env_kind: int = ENV_HOVER, wrapper: int = WRAP_NONE,
                 cfg: OracleCfg | None = None):
        self.cfg = cfg or default_cfg(env_kind, wrapper)
        self.s = OracleEnv()

    def reset_with(self, init12, target3):
        i12 = np.ascontiguousarray(init12, dtype=np.float32)
        t3 = np.ascontiguousarray(target3, dtype=np.float32)
        obs = np.zeros(12, np.float32)
        lib().oracle_env_reset(C.byref(self.cfg), C.byref(self.s), _fp(i12), _fp(t3), _fp(obs))
        return obs

    def relpos_obs(self, obs12):
        """RelPosActWrapper.observation of a base observation (wrappers.py:23-24)."""
        o12 = np.ascontiguousarray(obs12, dtype=np.float32)
        o7 = np.zeros(7, np.float32)
        lib().oracle_relpos_obs(C.byref(self.s), _fp(o12), _fp(o7))
        return o7

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float32)
        out = OracleStepOut()
        lib().oracle_env_step(C.byref(self.cfg), C.byref(self.s), _fp(a), C.byref(out))
        return out

    # state accessors -------------------------------------------------------------------
    @property
    def qpos(self):
        return np.array(self.s.qpos[:], dtype=np.float64)

    @property
    def qvel(self):
        return np.array(self.s.qvel[:], dtype=np.float64)

    @property
    def rate_int(self):
        return np.array(self.s.rate_int[:], dtype=np.float64)

    def set_full_state(self, qpos, qvel, voltage, target, step_count, rate_int=(0, 0, 0),
                       state12=None, prev_action=(0, 0, 0, 0)):
        self.s.qpos[:] = [float(x) for x in qpos]
        self.s.qvel[:] = [float(x) for x in qvel]
        self.s.voltage = float(voltage)
        self.s.target[:] = [float(x) for x in np.asarray(target, np.float32)]
        self.s.step_count = int(step_count)
        self.s.rate_int[:] = [float(x) for x in rate_int]
        self.s.prev_action[:] = [float(x) for x in np.asarray(prev_action, np.float32)]
        if state12 is None:
            obs = np.zeros(12, np.float32)
            lib().oracle_get_obs(C.byref(self.cfg), C.byref(self.s), _fp(obs))
        else:
            self.s.state12[:] = [float(x) for x in np.asarray(state12, np.float32)]


def out_to_dict(o: OracleStepOut) -> dict:
    return dict(obs=np.array(o.obs[:], np.float32), reward=float(o.reward),
                terminated=bool(o.terminated), truncated=bool(o.truncated),
                state12=np.array(o.state12[:], np.float32),
                motor_commands=np.array(o.motor_commands[:], np.float64),
                voltage=float(o.voltage), voltage_scale=float(o.voltage_scale),
                env_action=np.array(o.env_action[:], np.float32), obs7=np.array(o.obs7[:], np.float32))


class BraxEnv:
    """One brax-compat reference env (QuadHoverBraxEnv / JaxMJXQuadBraxEnv) under brax's
    EpisodeWrapper + AutoResetWrapper (see oracle/brax_oracle.c)."""

    def __init__(self, kind: int = ENV_BRAX_HOVER, episode_length: int = 500):
        self.cfg = OracleBraxCfg()
        lib().oracle_brax_default_cfg(kind, C.byref(self.cfg))
        self.cfg.episode_length = int(episode_length)
        self.s = OracleBraxEnv()

    def draw(self, seed: int, gid: int, episode: int):
        u = np.zeros(21, np.float32)
        lib().oracle_brax_reset_draw(C.byref(self.cfg), seed, gid, episode, _fp(u))
        return u

    def reset_with(self, u21):
        u = np.ascontiguousarray(u21, dtype=np.float32)
        obs = np.zeros(21, np.float32)
        lib().oracle_brax_reset(C.byref(self.cfg), C.byref(self.s), _fp(u), _fp(obs))
        return obs

    def step(self, action, auto_reset: bool = True) -> dict:
        a = np.ascontiguousarray(action, dtype=np.float32)
        o = OracleBraxOut()
        lib().oracle_brax_step(C.byref(self.cfg), C.byref(self.s), _fp(a), int(auto_reset), C.byref(o))
        return dict(obs=np.array(o.obs[:], np.float32), terminal_obs=np.array(o.terminal_obs[:], np.float32),
                    reward=float(o.reward), terminated=bool(o.terminated), truncated=bool(o.truncated),
                    motor_commands=np.array(o.motor_commands[:]), target=np.array(o.target[:], np.float32))
