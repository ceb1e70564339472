"""Policy export / import in the formats the reference's consumers load.

``save_sb3_zip`` writes a Stable-Baselines3 ``PPO.save`` archive of a policy trained here, so the
reference's ``PPO.load(path, device="cpu")`` call sites -- evaluate.py:309/459/628,
debug_training.py:94, ros2 policy_node.py:56 -- run it unchanged. Archive members (SB3
``save_util.save_to_zip_file``):

  data                      JSON of the algorithm attributes; entries SB3 cannot express in
                            JSON carry ``":serialized:"`` pickles (``json_to_data``): the policy
                            class, ``policy_kwargs`` (holds ``nn.ReLU``) and the two spaces
  policy.pth                ``ActorCriticPolicy.state_dict()`` (names already SB3's)
  policy.optimizer.pth      Adam state in SB3's parameter order (log_std first, see below)
  _stable_baselines3_version
  system_info.txt

The pickles reference classes by module path only (``stable_baselines3.common.policies.
ActorCriticPolicy``, ``gymnasium.spaces.box.Box``, ``torch.nn.modules.activation.ReLU``,
``numpy.dtype`` / ``numpy.array``), built here with stand-ins because neither SB3 nor gymnasium
is installed; Box state is the attribute dict gymnasium's ``Space.__setstate__`` restores, with
arrays rebuilt through ``numpy.array(list, dtype)`` so the pickle loads under numpy 1.x and 2.x.
Parity with a real SB3 install is unpinned (absent here); ``tests/test_export.py`` checks the
archive structure, the opcode-level pickle contents and the weights round trip.

``load_sb3_policy`` reads a reference-trained archive's ``policy.pth`` (``torch.load(...,
weights_only=True)``; nothing in the archive is unpickled) into an ``ActorCritic``.

``save_brax_params`` writes what brax's ``model.save_params`` writes for ``ppo.train``'s result
(train_brax_ppo.py:580-581, :624-625): a pickle of ``(RunningStatisticsState, policy, value)``
with flax-style ``{"params": {"hidden_i": {"kernel": [in, out], "bias"}}}`` trees (numpy leaves),
for the brax-profile learner (ppo/brax_ppo.py); ``brax.io.model.load_params`` and
evaluate_brax_ppo.py's ``make_inference_fn(...)(params)`` consume it. ``load_brax_params`` reads such
files back through an allow-list unpickler (numpy arrays and that one class only).
"""
from __future__ import annotations

import base64
import io
import json
import pickle
import platform
import sys
import types
import zipfile
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from .ppo.policy import ActorCritic

SB3_VERSION = "2.3.2"
_PICKLE_PROTOCOL = 4

# SB3 ActorCriticPolicy.parameters() order: the root's own log_std first, then mlp_extractor
# (policy_net then value_net), action_net, value_net (module registration order in
# ActorCriticPolicy._build / MlpExtractor.__init__)
SB3_PARAM_ORDER = ("log_std",
                   "mlp_extractor.policy_net.0.weight", "mlp_extractor.policy_net.0.bias",
                   "mlp_extractor.policy_net.2.weight", "mlp_extractor.policy_net.2.bias",
                   "mlp_extractor.value_net.0.weight", "mlp_extractor.value_net.0.bias",
                   "mlp_extractor.value_net.2.weight", "mlp_extractor.value_net.2.bias",
                   "action_net.weight", "action_net.bias", "value_net.weight", "value_net.bias")


# ---- pickles that reference third-party classes by path ------------------------------------
class _ArrayRef:
    """Pickles as ``numpy.array(values, dtype)`` (loadable by numpy 1.x and 2.x)."""

    def __init__(self, a: np.ndarray):
        self.values = np.asarray(a).tolist()
        self.dtype = str(np.asarray(a).dtype)

    def __reduce__(self):
        return (np.array, (self.values, self.dtype))


def _stand_in(module: str, name: str):
    """The real class if its package is installed, else a stand-in pickled by the same path."""
    try:
        return getattr(__import__(module, fromlist=[name]), name)
    except ImportError:
        return type(name, (), {"__module__": module, "__qualname__": name, "_stand_in": True})


class _FakeModules:
    """Temporarily install stand-in classes as `module.name` so pickle can reference them.
    Real (installed) classes are left alone; only modules created here are touched/removed."""

    def __init__(self, classes):
        self.classes = [c for c in classes if getattr(c, "_stand_in", False)]
        self.added = []

    def __enter__(self):
        for cls in self.classes:
            parts = cls.__module__.split(".")
            for i in range(1, len(parts) + 1):
                mod = ".".join(parts[:i])
                if mod not in sys.modules:
                    sys.modules[mod] = types.ModuleType(mod)
                    self.added.append(mod)
            if cls.__module__ not in self.added:
                raise RuntimeError(f"{cls.__module__} is partly installed; cannot stand in for it")
            setattr(sys.modules[cls.__module__], cls.__qualname__, cls)
        return self

    def __exit__(self, *exc):
        for mod in reversed(self.added):
            sys.modules.pop(mod, None)
        return False


_POLICY_CLS = _stand_in("stable_baselines3.common.policies", "ActorCriticPolicy")
_BOX_CLS = _stand_in("gymnasium.spaces.box", "Box")
_RSS_CLS = _stand_in("brax.training.acme.running_statistics", "RunningStatisticsState")


def _box(low: np.ndarray, high: np.ndarray):
    low = np.asarray(low, np.float32)
    high = np.asarray(high, np.float32)
    if not getattr(_BOX_CLS, "_stand_in", False):  # gymnasium installed: the real space
        return _BOX_CLS(low=low, high=high, dtype=np.float32)
    b = _BOX_CLS.__new__(_BOX_CLS)
    # gymnasium.spaces.Box attributes (restored by Space.__setstate__ / Box.__setstate__)
    b.__dict__.update({
        "dtype": np.dtype(np.float32), "_shape": tuple(low.shape),
        "low": _ArrayRef(low), "high": _ArrayRef(high),
        "bounded_below": _ArrayRef(np.isfinite(low)), "bounded_above": _ArrayRef(np.isfinite(high)),
        "low_repr": _short_repr(low), "high_repr": _short_repr(high), "_np_random": None})
    return b


def _short_repr(a: np.ndarray) -> str:
    return str(a.flat[0]) if a.size and np.all(a == a.flat[0]) else str(a)


def _serialized(obj, classes, readable: dict) -> dict:
    with _FakeModules(classes):
        raw = pickle.dumps(obj, protocol=_PICKLE_PROTOCOL)
    return {":type:": readable.pop(":type:"), ":serialized:": base64.b64encode(raw).decode(),
            **readable}


# ---- SB3 archive ------------------------------------------------------------------------------
def _sb3_data(cfg, num_timesteps: int, n_envs: int, obs_low, obs_high, act_low, act_high,
              net_arch, batch_size: int) -> dict:
    policy_kwargs = {"net_arch": list(net_arch), "activation_fn": nn.ReLU}
    return {
        "policy_class": _serialized(_POLICY_CLS, [_POLICY_CLS], {
            ":type:": "<class 'abc.ABCMeta'>", "__module__": "stable_baselines3.common.policies",
            "__doc__": "Policy class for actor-critic algorithms (has both policy and value prediction)."}),
        "verbose": 1,
        "policy_kwargs": _serialized(policy_kwargs, [], {
            ":type:": "<class 'dict'>", "net_arch": list(net_arch),
            "activation_fn": "<class 'torch.nn.modules.activation.ReLU'>"}),
        "num_timesteps": int(num_timesteps),
        "_total_timesteps": int(num_timesteps),
        "_num_timesteps_at_start": 0,
        "seed": None,
        "action_noise": None,
        "learning_rate": float(cfg.learning_rate),
        "tensorboard_log": None,
        "_last_obs": None,
        "_last_episode_starts": None,
        "_last_original_obs": None,
        "_episode_num": 0,
        "use_sde": False,
        "sde_sample_freq": -1,
        "_current_progress_remaining": 0.0,
        "_stats_window_size": 100,
        "_n_updates": 0,
        "observation_space": _serialized(_box(obs_low, obs_high), [_BOX_CLS], {
            ":type:": "<class 'gymnasium.spaces.box.Box'>", "dtype": "float32",
            "_shape": list(np.shape(obs_low)), "low": np.asarray(obs_low, np.float32).tolist(),
            "high": np.asarray(obs_high, np.float32).tolist(), "_np_random": None}),
        "action_space": _serialized(_box(act_low, act_high), [_BOX_CLS], {
            ":type:": "<class 'gymnasium.spaces.box.Box'>", "dtype": "float32",
            "_shape": list(np.shape(act_low)), "low": np.asarray(act_low, np.float32).tolist(),
            "high": np.asarray(act_high, np.float32).tolist(), "_np_random": None}),
        "n_envs": int(n_envs),
        "n_steps": int(cfg.n_steps),
        "gamma": float(cfg.gamma),
        "gae_lambda": float(cfg.gae_lambda),
        "ent_coef": float(cfg.ent_coef),
        "vf_coef": float(cfg.vf_coef),
        "max_grad_norm": float(cfg.max_grad_norm),
        "rollout_buffer_kwargs": {},
        "batch_size": int(batch_size),
        "n_epochs": int(cfg.n_epochs),
        "clip_range": float(cfg.clip_range),
        "clip_range_vf": None,
        "normalize_advantage": bool(cfg.normalize_advantage),
        "target_kl": None,
    }


def _sb3_optimizer_state(policy: ActorCritic, opt: Optional[torch.optim.Optimizer], cfg) -> dict:
    names = [n for n, _ in policy.named_parameters()]
    params = dict(policy.named_parameters())
    state = {}
    if opt is not None:
        ours = opt.state_dict()
        idx_of = {n: i for i, n in enumerate(names)}  # our Adam was built from policy.parameters()
        for j, n in enumerate(SB3_PARAM_ORDER):
            st = ours["state"].get(idx_of[n])
            if st:
                state[j] = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
    group = {"lr": float(cfg.learning_rate), "betas": (0.9, 0.999), "eps": float(cfg.adam_eps),
             "weight_decay": 0, "amsgrad": False, "maximize": False, "foreach": None,
             "capturable": False, "differentiable": False, "fused": None,
             "params": list(range(len(SB3_PARAM_ORDER)))}
    assert set(params) == set(SB3_PARAM_ORDER)
    return {"state": state, "param_groups": [group]}


def save_sb3_zip(path: str, policy: ActorCritic, optimizer: Optional[torch.optim.Optimizer] = None,
                 cfg=None, num_timesteps: int = 0, n_envs: int = 16, batch_size: int = 128,
                 obs_low=None, obs_high=None) -> str:
    """Write `path` (".zip" appended if missing) as an SB3 PPO archive of `policy`."""
    from .ppo.ppo import PPOConfig
    cfg = cfg or PPOConfig()
    if not path.endswith(".zip"):
        path += ".zip"
    obs_dim = policy.mlp_extractor.policy_net[0].in_features
    act_dim = policy.action_net.out_features
    obs_low = np.full(obs_dim, -1.0, np.float32) if obs_low is None else obs_low
    obs_high = np.full(obs_dim, 1.0, np.float32) if obs_high is None else obs_high
    net_arch = [m.out_features for m in policy.mlp_extractor.policy_net if isinstance(m, nn.Linear)]
    data = _sb3_data(cfg, num_timesteps, n_envs, obs_low, obs_high, np.full(act_dim, -1.0, np.float32),
                     np.full(act_dim, 1.0, np.float32), net_arch, batch_size)
    sd = {k: v.detach().cpu().clone() for k, v in policy.state_dict().items()}
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("data", json.dumps(data, indent=4))
        for name, obj in (("policy.pth", sd), ("policy.optimizer.pth", _sb3_optimizer_state(policy, optimizer, cfg))):
            buf = io.BytesIO()
            torch.save(obj, buf)
            z.writestr(name, buf.getvalue())
        z.writestr("_stable_baselines3_version", SB3_VERSION)
        z.writestr("system_info.txt", f"- OS: {platform.platform()}\n- Python: {platform.python_version()}\n"
                                      f"- Stable-Baselines3: {SB3_VERSION}\n- PyTorch: {torch.__version__}\n"
                                      f"- Numpy: {np.__version__}\n- exported by uav_reinforcement_learning_control_amd\n")
    return path


def load_sb3_policy(path: str, device="cpu") -> ActorCritic:
    """ActorCritic from an SB3 PPO archive (the reference's train.py output). Only the JSON
    `data` and `policy.pth` (weights_only=True) are read; no pickle in the archive is loaded."""
    with zipfile.ZipFile(path) as z:
        data = json.loads(z.read("data"))
        sd = torch.load(io.BytesIO(z.read("policy.pth")), map_location="cpu", weights_only=True)
    pk = data.get("policy_kwargs", {})
    arch = pk.get("net_arch", [64, 64])
    if isinstance(arch, dict):
        arch = arch.get("pi", [64, 64])
    obs_dim = sd["mlp_extractor.policy_net.0.weight"].shape[1]
    act_dim = sd["action_net.weight"].shape[0]
    act = str(pk.get("activation_fn", "ReLU"))
    if "ReLU" not in act:
        raise ValueError(f"only ReLU policies are supported, archive has {act}")
    pol = ActorCritic(obs_dim, act_dim, tuple(arch))
    pol.load_state_dict(sd, strict=True)
    return pol.to(device)


# ---- brax params ("ppo_params.msgpack") -------------------------------------------------------
def _tree_refs(tree):
    if isinstance(tree, dict):
        return {k: _tree_refs(v) for k, v in tree.items()}
    return _ArrayRef(np.asarray(tree, np.float32))


def save_brax_params(path: str, params) -> str:
    """brax ``model.save_params(path, (normalizer, policy, value))`` for BraxPPO.params()."""
    norm, pol, val = params
    if getattr(_RSS_CLS, "_stand_in", False):
        rss = _RSS_CLS.__new__(_RSS_CLS)
        rss.__dict__.update({k: _ArrayRef(np.asarray(norm[k], np.float32))
                             for k in ("mean", "std", "count", "summed_variance")})
    else:  # brax installed: the real flax dataclass
        rss = _RSS_CLS(mean=np.asarray(norm["mean"], np.float32), std=np.asarray(norm["std"], np.float32),
                       count=np.asarray(norm["count"], np.float32),
                       summed_variance=np.asarray(norm["summed_variance"], np.float32))
    with _FakeModules([_RSS_CLS]):
        raw = pickle.dumps((rss, _tree_refs(pol), _tree_refs(val)), protocol=_PICKLE_PROTOCOL)
    with open(path, "wb") as f:
        f.write(raw)
    return path


class _BraxParamsUnpickler(pickle.Unpickler):
    class _RSS:
        def __setstate__(self, state):
            self.__dict__.update(state)

    def find_class(self, module, name):
        if (module, name) == ("brax.training.acme.running_statistics", "RunningStatisticsState"):
            return self._RSS
        if (module, name) in (("numpy", "array"), ("numpy", "dtype"), ("copyreg", "__newobj__")):
            import copyreg
            return copyreg.__newobj__ if module == "copyreg" else getattr(np, name)
        if (module, name) in (("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                              ("numpy", "ndarray")):
            return np.core.multiarray._reconstruct if name == "_reconstruct" else np.ndarray
        raise pickle.UnpicklingError(f"refusing {module}.{name} in a params file")


def load_brax_params(path: str):
    """(normalizer dict, policy tree, value tree) from a params file with numpy leaves."""
    with open(path, "rb") as f:
        rss, pol, val = _BraxParamsUnpickler(f).load()
    norm = {k: np.asarray(getattr(rss, k)) for k in ("mean", "std", "count", "summed_variance")}
    return norm, pol, val
