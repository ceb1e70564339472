"""ctypes binding of libquadenv.so (the C ABI in include/quadenv.h).

The library is built in-tree by ``__graft_entry__.build()`` (``csrc/Makefile`` -> ``_lib/``).
There is no fallback: if the library is missing or fails to load, every env constructor raises.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "_lib", "libquadenv.so")
if os.environ.get("QUADENV_LIB"):  # A/B and ablation builds of the same library (tools/*_variants.sh)
    LIB_PATH = os.environ["QUADENV_LIB"]
CSRC = os.path.join(_PKG, "csrc")

QUAD_OK, QUAD_EINVAL, QUAD_EHIP, QUAD_ENOMEM, QUAD_EMODEL = 0, -1, -2, -3, -4
QUAD_ADV_PRECOMPUTED = 2  # QuadPPOBatch.normalize_advantage: quad_ppo_adv_stats already ran
QUAD_ADV_GIVEN = 3        # ... : the sums are in QuadPPOBatch.adv_sums (quad_ppo_adv_stats_epoch)
ADV_SUM_DOUBLES = 512     # QUAD_ADV_SUM_DOUBLES: one minibatch's block sums
ENV_HOVER, ENV_TRAJ, ENV_BRAX_HOVER, ENV_BRAX_TRAJ = 0, 1, 2, 3
WRAP_NONE, WRAP_CTBR, WRAP_RELPOS, WRAP_CTBR_RELPOS = 0, 1, 2, 3
ABI_VERSION = 5


class QuadCfg(C.Structure):
    _fields_ = [
        ("env_kind", C.c_int32), ("wrapper", C.c_int32), ("max_episode_steps", C.c_int32),
        ("auto_reset", C.c_int32),
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
        ("timestep", C.c_double), ("gravity", C.c_double * 3), ("density", C.c_double),
        ("viscosity", C.c_double),
        ("reset_noise", C.c_float), ("reward_pos_coef", C.c_float),
        ("reward_action_coef", C.c_float), ("vel_limit", C.c_float),
        ("traj_center", C.c_float * 3), ("traj_amp", C.c_float * 3), ("traj_freq", C.c_float * 3),
        ("traj_duration", C.c_float),
        ("spline_center_low", C.c_float * 3), ("spline_center_high", C.c_float * 3),
        ("spline_amp", C.c_float * 3), ("spline_duration", C.c_float),
    ]


class QuadStateSoA(C.Structure):
    _fields_ = [("qpos", C.c_void_p), ("qvel", C.c_void_p), ("voltage", C.c_void_p),
                ("target", C.c_void_p), ("rate_int", C.c_void_p), ("step_count", C.c_void_p),
                ("episode", C.c_void_p), ("prev_action", C.c_void_p)]


class QuadStepOut(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("reward", C.c_void_p), ("terminated", C.c_void_p),
                ("truncated", C.c_void_p), ("terminal_obs", C.c_void_p),
                ("motor_commands", C.c_void_p), ("voltage_scale", C.c_void_p),
                ("state12", C.c_void_p), ("target_info", C.c_void_p)]


class QuadPolicyParams(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("pi_w0", "pi_b0", "pi_w1", "pi_b1", "act_w", "act_b",
                                          "vf_w0", "vf_b0", "vf_w1", "vf_b1", "val_w", "val_b",
                                          "log_std")]


class QuadWaypoints(C.Structure):
    _fields_ = [("points", C.c_void_p), ("counts", C.c_void_p), ("set_of", C.c_void_p),
                ("max_points", C.c_int32), ("reach_radius", C.c_float)]


class QuadWaypointState(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("wp_idx", "reached", "laps", "steps", "status", "total_reward")]


POLICY_STAT_SLOTS = 1024


class QuadRolloutPost(C.Structure):
    _fields_ = [("reward", C.c_void_p), ("terminated", C.c_void_p), ("truncated", C.c_void_p),
                ("terminal_obs", C.c_void_p), ("buf_rew", C.c_void_p), ("last_start", C.c_void_p),
                ("ep_ret", C.c_void_p), ("ep_len", C.c_void_p), ("stats", C.c_void_p),
                ("rows", C.c_int32), ("gamma", C.c_float)]


class QuadPolicyAct(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("actions_env", C.c_void_p), ("actions", C.c_void_p),
                ("log_prob", C.c_void_p), ("value", C.c_void_p), ("obs_copy", C.c_void_p),
                ("last_start", C.c_void_p), ("episode_starts", C.c_void_p),
                ("cursor", C.c_void_p), ("rows", C.c_int32), ("deterministic", C.c_int32),
                ("seed", C.c_uint64), ("env_id_base", C.c_uint64),
                ("epilogue", C.POINTER(QuadRolloutPost))]


# every symbol include/quadenv.h declares (checked by tests/test_abi.py)
EXPORTS = ("quad_abi_version", "quad_last_error", "quad_default_cfg", "quad_create",
           "quad_destroy", "quad_num_envs", "quad_seed", "quad_reset", "quad_step", "quad_step_range", "quad_observe", "quad_terminated", "quad_step_random",
           "quad_mem_floor",
           "quad_kernel_form", "quad_random_actions", "quad_get_state", "quad_set_state", "quad_gae",
           "quad_policy_packed_floats", "quad_policy_pack", "quad_policy_act", "quad_rollout_post", "quad_rollout",
           "quad_waypoints_begin", "quad_waypoints_update", "quad_ppo_workspace_bytes", "quad_ppo_grad",
           "quad_ppo_grad_form", "quad_ppo_hidden", "quad_ppo_adv_stats", "quad_ppo_adv_stats_epoch", "quad_permutation", "quad_adam_workspace_bytes",
           "quad_clip_adam")


class QuadRollout(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("obs_copy", "actions", "log_prob", "value", "episode_starts",
                                          "rewards", "last_obs", "last_start", "ep_ret", "ep_len",
                                          "stats")] + \
               [("rows", C.c_int32), ("t0", C.c_int32), ("steps", C.c_int32), ("deterministic", C.c_int32),
                ("seed", C.c_uint64), ("gamma", C.c_float)]


class QuadPolicyGrads(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("pi_w0", "pi_b0", "pi_w1", "pi_b1", "act_w", "act_b",
                                          "vf_w0", "vf_b0", "vf_w1", "vf_b1", "val_w", "val_b",
                                          "log_std")]


class QuadPPOBatch(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("obs", "actions", "log_prob", "advantages", "returns", "index")] + \
               [("batch", C.c_int32), ("normalize_advantage", C.c_int32), ("clip_range", C.c_float),
                ("ent_coef", C.c_float), ("vf_coef", C.c_float), ("stats", C.c_void_p), ("adv_sums", C.c_void_p)]


ADAM_MAX_TENSORS = 16


class QuadAdam(C.Structure):
    _fields_ = [(n, C.c_void_p * ADAM_MAX_TENSORS) for n in ("params", "grads", "exp_avg", "exp_avg_sq", "step")] + \
               [("numel", C.c_int32 * ADAM_MAX_TENSORS), ("count", C.c_int32), ("max_grad_norm", C.c_float),
                ("lr", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_double)]


class QuadError(RuntimeError):
    pass


_lib = None


def _declare(L):
    vp, i32, u32, u64 = C.c_void_p, C.c_int32, C.c_uint32, C.c_uint64
    L.quad_abi_version.restype = C.c_int
    L.quad_last_error.restype = C.c_char_p
    L.quad_default_cfg.argtypes = [i32, i32, C.POINTER(QuadCfg)]
    L.quad_create.argtypes = [C.POINTER(QuadCfg), i32, u64, u64, i32, C.POINTER(vp)]
    L.quad_destroy.argtypes = [vp]
    L.quad_destroy.restype = None
    L.quad_num_envs.argtypes = [vp]
    L.quad_num_envs.restype = i32
    L.quad_seed.argtypes = [vp, u64, vp]
    L.quad_reset.argtypes = [vp, vp, vp, vp]
    L.quad_step.argtypes = [vp, vp, C.POINTER(QuadStepOut), vp]
    L.quad_step_range.argtypes = [vp, i32, i32, vp, C.POINTER(QuadStepOut), vp]
    L.quad_observe.argtypes = [vp, vp, vp, vp]
    L.quad_terminated.argtypes = [vp, vp, i32, vp, vp]
    L.quad_step_random.argtypes = [vp, u32, i32, C.POINTER(QuadStepOut), vp, vp]
    if hasattr(L, "quad_mem_floor"):  # (added in round 6 as a backward-compatible entry; A/B tools load older builds)
        L.quad_mem_floor.argtypes = [vp, vp, C.POINTER(QuadStepOut), vp]
    L.quad_kernel_form.argtypes = [vp]
    L.quad_kernel_form.restype = i32
    L.quad_random_actions.argtypes = [vp, u32, vp, vp]
    L.quad_get_state.argtypes = [vp, C.POINTER(QuadStateSoA), i32, vp]
    L.quad_set_state.argtypes = [vp, C.POINTER(QuadStateSoA), i32, vp]
    L.quad_gae.argtypes = [vp, vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp, vp]
    L.quad_policy_packed_floats.argtypes = []
    L.quad_policy_packed_floats.restype = i32
    L.quad_policy_pack.argtypes = [C.POINTER(QuadPolicyParams), vp, vp]
    L.quad_policy_act.argtypes = [vp, C.POINTER(QuadPolicyAct), i32, vp]
    L.quad_rollout_post.argtypes = [vp, C.POINTER(QuadRolloutPost), vp, i32, vp]
    L.quad_rollout.argtypes = [vp, vp, C.POINTER(QuadRollout), vp]
    L.quad_waypoints_begin.argtypes = [vp, C.POINTER(QuadWaypoints), C.POINTER(QuadWaypointState), vp, vp]
    L.quad_waypoints_update.argtypes = [vp, C.POINTER(QuadWaypoints), C.POINTER(QuadWaypointState),
                                        vp, vp, vp, vp, vp]
    L.quad_ppo_workspace_bytes.argtypes = [i32]
    L.quad_ppo_workspace_bytes.restype = C.c_int64
    L.quad_ppo_grad_form.argtypes = []
    L.quad_ppo_grad_form.restype = i32
    L.quad_permutation.argtypes = [C.c_int64, u64, vp, vp]
    L.quad_ppo_grad.argtypes = [C.POINTER(QuadPolicyParams), C.POINTER(QuadPPOBatch), C.POINTER(QuadPolicyGrads),
                                vp, C.c_int64, vp]
    L.quad_ppo_hidden.argtypes = [C.POINTER(QuadPolicyParams), C.POINTER(QuadPPOBatch), C.POINTER(QuadPolicyGrads),
                                  vp, vp, C.c_int64, vp]
    L.quad_ppo_adv_stats.argtypes = [C.POINTER(QuadPPOBatch), vp, C.c_int64, vp]
    L.quad_ppo_adv_stats_epoch.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, vp]
    L.quad_adam_workspace_bytes.argtypes = [C.POINTER(QuadAdam)]
    L.quad_adam_workspace_bytes.restype = C.c_int64
    L.quad_clip_adam.argtypes = [C.POINTER(QuadAdam), vp, C.c_int64, vp]
    for n in ("quad_clip_adam", "quad_ppo_grad", "quad_ppo_hidden", "quad_ppo_adv_stats", "quad_ppo_adv_stats_epoch", "quad_default_cfg", "quad_create", "quad_seed", "quad_reset", "quad_step", "quad_step_range", "quad_observe", "quad_terminated", "quad_step_random",
              "quad_random_actions", "quad_get_state", "quad_set_state", "quad_gae",
              "quad_policy_pack", "quad_policy_act", "quad_rollout_post", "quad_rollout",
              "quad_waypoints_begin", "quad_waypoints_update"):
        getattr(L, n).restype = C.c_int


def lib():
    """Load libquadenv.so; raise loudly if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QuadError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
                            f"g.build()'` (or make -C {CSRC}) to build the HIP extension")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        if L.quad_abi_version() != ABI_VERSION:
            raise QuadError("libquadenv.so ABI version mismatch; rebuild it")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != QUAD_OK:
        msg = lib().quad_last_error().decode(errors="replace")
        raise QuadError(f"{what} failed ({rc}): {msg}")


def default_cfg(env_kind: int = ENV_HOVER, wrapper: int = WRAP_NONE) -> QuadCfg:
    cfg = QuadCfg()
    check(lib().quad_default_cfg(env_kind, wrapper, C.byref(cfg)), "quad_default_cfg")
    return cfg
