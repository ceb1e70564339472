"""Learning-level pin of row P: reproduce the reference's HPO trial 31 -- TEST INFRASTRUCTURE.

The reference's only evidence about learning is its Optuna record (``tests/golden/hpo_trial31.json``,
written by ``tools/extract_hpo_curve.py`` from ``optuna_full.db``): the run ``optimize.py`` makes
with ``train.py``'s hyperparameters scored 7.1, 19.9, 262.7, 419.1, 399.4, 466.8, 414.8, 418.3,
429.0, 477.4 at 50k, 100k, ..., 500k env steps. This harness runs that configuration

  * HoverEnv + RateControlWrapper (``optimize.py:26``), ``make_vec_env(n_envs=8)`` (``:244``),
  * SB3 PPO with ``train.py:50-68``'s parameters (n_steps 1024, batch 128, 20 epochs, ReLU
    [128, 128]; the batch clamp of ``optimize.py:135-144`` keeps 128: 8 x 1024 % 128 == 0),
  * ``TrialEvalCallback`` every 50,000 env steps (``eval_freq // n_envs`` = 6,250 vec steps,
    ``optimize.py:161-167,254``): 10 deterministic episodes over 5 eval envs, mean episode return,
  * until 10 evaluations have been made (``learn(500_000)``, ``optimize.py:244,172``),

along two paths:

  ``gpu``  the product: QuadVecEnv (HIP env kernels, CTBR fused) + ppo.PPO (quad_rollout MFMA
           rollout, quad_gae, quad_ppo_grad minibatch gradient, quad_clip_adam), 8 envs;
  ``cpu``  the checker: 8 float64 oracle envs stepped one after another (DummyVecEnv order) and a
           torch-CPU SB3 PPO restatement (ActorCritic + ppo_loss, torch.randperm shuffles,
           clip_grad_norm_, Adam) -- the oracle is used here as test infrastructure only.

Evaluation timing follows SB3: the callback fires at vec step 6,250 k, which falls inside a rollout,
so the policy evaluated is the one that rollout is being collected with (the parameters after the
previous update). Here the evaluation runs after that rollout's collection and before its update:
the same parameters. The 5 eval envs x 2 episodes each of ``evaluate_policy`` become 10 independent
episodes from fresh resets (the episodes are i.i.d. draws of the reset distribution either way).

    python tests/hpo_repro.py --path gpu --seeds 0 1 2 3 4 --out gpurun_out/hpo_gpu.json
    python tests/hpo_repro.py --path cpu --seeds 0 --out /tmp/hpo_cpu_0.json
    python tests/hpo_repro.py --combine gpu.json cpu_*.json --out profiles/r06/hpo_repro.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden", "hpo_trial31.json")


def load_anchor() -> dict:
    with open(GOLDEN) as f:
        return json.load(f)


def ppo_config():
    """train.py:50-68 (= trial 31's decoded parameters)."""
    from uav_reinforcement_learning_control_amd.ppo import PPOConfig
    a = load_anchor()["params"]
    return PPOConfig(learning_rate=a["learning_rate"], n_steps=a["n_steps"], batch_size=a["batch_size"],
                     n_epochs=a["n_epochs"], gamma=1.0 - a["gamma_inv"], gae_lambda=a["gae_lambda"],
                     clip_range=a["clip_range"], ent_coef=a["ent_coef"])


def eval_points() -> list:
    return list(load_anchor()["eval_timesteps"])


def _progress(path: str, seed: int, steps: int, value: float, t0: float) -> None:
    print(f"  [{path} seed {seed}] {steps:7d} steps  eval {value:7.1f}  {time.perf_counter() - t0:7.1f} s", flush=True)


# ----------------------------------------------------------------------------------------------
# GPU path: the product
# ----------------------------------------------------------------------------------------------
WRAPPERS = {"RateControlWrapper": "RateControlWrapper", "none": None}


def run_gpu(seed: int, n_envs: int = 8, n_eval: int = 10, wrapper: str = "RateControlWrapper") -> dict:
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.evaluate import evaluate_episodes
    from uav_reinforcement_learning_control_amd.ppo import PPO
    dev = torch.device("cuda", 0)
    env = QuadVecEnv(n_envs, env="hover", wrapper=WRAPPERS[wrapper], device=dev, seed=seed)
    model = PPO(env, ppo_config(), seed=seed)
    if model._learner is None or not model._one_launch:
        raise RuntimeError("the GPU path must run the fused HIP rollout and learner")
    points, curve, lengths = eval_points(), [], []
    t0 = time.perf_counter()
    t_train = t_eval = 0.0
    updates = 0
    while len(curve) < len(points):
        model.collect_rollouts()
        while len(curve) < len(points) and model.num_timesteps >= points[len(curve)]:
            te = time.perf_counter()
            r = evaluate_episodes(model.policy, num_episodes=n_eval, wrapper=WRAPPERS[wrapper],
                                  device=dev, seed=1_000_003 * (seed + 1) + len(curve))
            t_eval += time.perf_counter() - te
            curve.append(r["mean_reward"])
            lengths.append(r["mean_length"])
            _progress("gpu", seed, model.num_timesteps, curve[-1], t0)
        if len(curve) == len(points):
            break  # learn(500_000)'s last update comes after the 10th evaluation
        tu = time.perf_counter()
        model.train()
        torch.cuda.synchronize(dev)
        t_train += time.perf_counter() - tu
        updates += 1
    env.close()
    return {"seed": seed, "curve": curve, "mean_length": lengths, "updates": updates,
            "optimizer_steps": updates * model.n_minibatches_per_epoch() * model.cfg.n_epochs,
            "env_steps": model.num_timesteps, "seconds": time.perf_counter() - t0,
            "train_seconds": t_train, "eval_seconds": t_eval}


# ----------------------------------------------------------------------------------------------
# CPU path: float64 oracle envs + torch-CPU SB3 PPO restatement (the checker)
# ----------------------------------------------------------------------------------------------
class _OracleVec:
    """make_vec_env(n) over oracle envs: DummyVecEnv order, auto-reset, terminal observations."""

    def __init__(self, n: int, seed: int, wrap: int):
        from oracle import oracle as O
        self.O = O
        self.cfg = O.default_cfg(O.ENV_HOVER, wrap)
        self.envs = [O.Env(cfg=self.cfg) for _ in range(n)]
        self.seed, self.episode = seed, [0] * n

    def reset(self) -> np.ndarray:
        return np.stack([e.reset_with(*self.O.reset_draw(self.cfg, self.seed, i, self.episode[i]))
                         for i, e in enumerate(self.envs)])

    def step(self, actions: np.ndarray):
        n = len(self.envs)
        obs = np.zeros((n, 12), np.float32)
        rew = np.zeros(n, np.float32)
        term, trunc = np.zeros(n, bool), np.zeros(n, bool)
        terminal = {}
        for i, e in enumerate(self.envs):
            o = e.step(actions[i])
            rew[i] = np.float32(o.reward)
            term[i], trunc[i] = bool(o.terminated), bool(o.truncated)
            if term[i] or trunc[i]:
                terminal[i] = np.array(o.obs[:], np.float32)
                self.episode[i] += 1
                obs[i] = e.reset_with(*self.O.reset_draw(self.cfg, self.seed, i, self.episode[i]))
            else:
                obs[i] = np.array(o.obs[:], np.float32)
        return obs, rew, term, trunc, terminal


def _evaluate_cpu(pol, seed: int, wrap: int, n_episodes: int = 10) -> tuple:
    """evaluate_policy(deterministic=True): n_episodes from fresh resets, mean episode return."""
    from oracle import oracle as O
    cfg = O.default_cfg(O.ENV_HOVER, wrap)
    envs = [O.Env(cfg=cfg) for _ in range(n_episodes)]
    obs = np.stack([e.reset_with(*O.reset_draw(cfg, seed, i, 0)) for i, e in enumerate(envs)])
    ret, length = np.zeros(n_episodes), np.zeros(n_episodes, np.int64)
    running = np.ones(n_episodes, bool)
    with torch.no_grad():
        while running.any():
            mean, _ = pol.forward_heads(torch.from_numpy(obs))
            a = mean.clamp(-1.0, 1.0).numpy()
            for i in np.nonzero(running)[0]:
                o = envs[i].step(a[i])
                ret[i] += float(np.float32(o.reward))
                length[i] += 1
                obs[i] = np.array(o.obs[:], np.float32)
                if o.terminated or o.truncated:
                    running[i] = False
    return float(ret.mean()), float(length.mean())


def run_cpu(seed: int, n_envs: int = 8, n_eval: int = 10, wrapper: str = "RateControlWrapper") -> dict:
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import ppo_loss
    torch.set_num_threads(1)  # optimize.py:249
    cfg = ppo_config()
    T, B = cfg.n_steps, cfg.batch_size
    torch.manual_seed(seed)
    pol = ActorCritic()
    opt = torch.optim.Adam(pol.parameters(), lr=cfg.learning_rate, eps=cfg.adam_eps)
    from oracle import oracle as O
    wrap = O.WRAP_CTBR if wrapper == "RateControlWrapper" else O.WRAP_NONE
    venv = _OracleVec(n_envs, seed, wrap)
    obs = venv.reset()
    start = np.ones(n_envs, np.float32)
    buf_obs, buf_act = torch.zeros(T, n_envs, 12), torch.zeros(T, n_envs, 4)
    buf_lp, buf_v, buf_r, buf_s = (torch.zeros(T, n_envs) for _ in range(4))
    points, curve, lengths = eval_points(), [], []
    num_timesteps, updates = 0, 0
    t0 = time.perf_counter()
    t_train = t_eval = 0.0
    while len(curve) < len(points):
        with torch.no_grad():  # OnPolicyAlgorithm.collect_rollouts
            for t in range(T):
                o = torch.from_numpy(obs)
                mean, v = pol.forward_heads(o)
                a = mean + pol.log_std.exp() * torch.randn_like(mean)
                buf_obs[t], buf_act[t], buf_lp[t], buf_v[t] = o, a, pol.log_prob(mean, a), v
                buf_s[t] = torch.from_numpy(start)
                obs, rew, term, trunc, terminal = venv.step(a.clamp(-1.0, 1.0).numpy())
                r = torch.from_numpy(rew)
                for i, to in terminal.items():  # TimeLimit bootstrap
                    if trunc[i] and not term[i]:
                        r[i] += cfg.gamma * pol.value(torch.from_numpy(to)[None])[0]
                buf_r[t] = r
                start = (term | trunc).astype(np.float32)
            last_v = pol.value(torch.from_numpy(obs))
        num_timesteps += T * n_envs
        while len(curve) < len(points) and num_timesteps >= points[len(curve)]:
            te = time.perf_counter()
            m, l = _evaluate_cpu(pol, 1_000_003 * (seed + 1) + len(curve), wrap)
            t_eval += time.perf_counter() - te
            curve.append(m)
            lengths.append(l)
            _progress("cpu", seed, num_timesteps, m, t0)
        if len(curve) == len(points):
            break
        tu = time.perf_counter()
        adv = torch.zeros(T, n_envs)  # RolloutBuffer.compute_returns_and_advantage
        acc = torch.zeros(n_envs)
        nxt_start = torch.from_numpy(start)
        for t in reversed(range(T)):
            nv, nnt = (last_v, 1.0 - nxt_start) if t == T - 1 else (buf_v[t + 1], 1.0 - buf_s[t + 1])
            delta = buf_r[t] + cfg.gamma * nv * nnt - buf_v[t]
            acc = delta + cfg.gamma * cfg.gae_lambda * nnt * acc
            adv[t] = acc
        ret = adv + buf_v
        M = T * n_envs
        flat = [buf_obs.view(M, 12), buf_act.view(M, 4), buf_lp.view(M), adv.view(M), ret.view(M)]
        for _ in range(cfg.n_epochs):  # PPO.train
            perm = torch.randperm(M)
            for s in range(0, M, B):
                idx = perm[s:s + B]
                loss = ppo_loss(pol, *[x[idx] for x in flat], cfg)[0]
                opt.zero_grad()
                loss.backward()
                torch.nn.utils.clip_grad_norm_(pol.parameters(), cfg.max_grad_norm)
                opt.step()
        t_train += time.perf_counter() - tu
        updates += 1
    return {"seed": seed, "curve": curve, "mean_length": lengths, "updates": updates,
            "optimizer_steps": updates * (T * n_envs // B) * cfg.n_epochs, "env_steps": num_timesteps,
            "seconds": time.perf_counter() - t0, "train_seconds": t_train, "eval_seconds": t_eval}


# ----------------------------------------------------------------------------------------------
def summarize(runs: dict) -> dict:
    """Per path: per-point mean / std / median over seeds, the final evaluations; GPU vs CPU
    agreement (|mean difference| <= 2 standard errors of the difference at every point, and a
    two-sided rank-sum test of the final points); the reference band (its last five evaluations)."""
    a = load_anchor()
    ref = a["eval_mean_reward"]
    band = (min(ref[5:]), max(ref[5:]))
    out = {"reference": {"eval_timesteps": a["eval_timesteps"], "eval_mean_reward": ref, "band_last5": band,
                         "source": a["source"]}}
    for path, rs in runs.items():
        C = np.array([r["curve"] for r in rs])
        finals = C[:, -1]
        last5 = C[:, 5:].mean(1)
        out[path] = {"seeds": [r["seed"] for r in rs], "curves": C.tolist(),
                     "mean": C.mean(0).tolist(), "std": C.std(0, ddof=1).tolist() if len(rs) > 1 else None,
                     "median": np.median(C, 0).tolist(), "final": finals.tolist(),
                     "median_final": float(np.median(finals)), "mean_last5": last5.tolist(),
                     "median_final_in_band": bool(band[0] <= float(np.median(finals)) <= band[1]),
                     "seconds_per_seed": statistics.mean(r["seconds"] for r in rs),
                     "train_seconds_per_seed": statistics.mean(r["train_seconds"] for r in rs),
                     "optimizer_steps": rs[0]["optimizer_steps"], "env_steps": rs[0]["env_steps"]}
    if "gpu" in runs and "cpu" in runs and len(runs["gpu"]) > 1 and len(runs["cpu"]) > 1:
        G, Cc = np.array(out["gpu"]["curves"]), np.array(out["cpu"]["curves"])
        se = np.sqrt(G.var(0, ddof=1) / len(G) + Cc.var(0, ddof=1) / len(Cc))
        d = G.mean(0) - Cc.mean(0)
        from scipy.stats import mannwhitneyu
        p_final = float(mannwhitneyu(G[:, -1], Cc[:, -1], alternative="two-sided").pvalue)
        p_last5 = float(mannwhitneyu(G[:, 5:].mean(1), Cc[:, 5:].mean(1), alternative="two-sided").pvalue)
        out["gpu_vs_cpu"] = {"mean_diff": d.tolist(), "se_diff": se.tolist(),
                             "within_2se": [bool(abs(x) <= 2 * s) for x, s in zip(d, se)],
                             "mannwhitney_p_final": p_final, "mannwhitney_p_last5_mean": p_last5}
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--path", choices=["gpu", "cpu"])
    ap.add_argument("--seeds", type=int, nargs="+", default=[0])
    ap.add_argument("--n-envs", type=int, default=8,
                    help="training envs (optimize.py's --n-envs: default 8; optimize.sh passes 16, train.py uses 16)")
    ap.add_argument("--permutation", choices=["feistel", "randperm"], default="feistel",
                    help="GPU path's epoch permutation: quad_permutation (the product) or torch.randperm")
    ap.add_argument("--wrapper", choices=sorted(WRAPPERS), default="RateControlWrapper",
                    help="optimize.py:26's wrapper_cls (RateControlWrapper) or the bare HoverEnv")
    ap.add_argument("--combine", nargs="+", help="per-path result files to summarize")
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    if a.combine:
        runs = {}
        for fn in a.combine:
            with open(fn) as f:
                d = json.load(f)
            key = d["path"] if d.get("wrapper", "RateControlWrapper") == "RateControlWrapper" else f'{d["path"]}_{d["wrapper"]}'
            if d.get("permutation", "feistel") != "feistel":
                key += "_" + d["permutation"]
            if d.get("n_envs", 8) != 8:
                key += f'_{d["n_envs"]}envs'
            runs.setdefault(key, []).extend(d["runs"])
        for rs in runs.values():
            rs.sort(key=lambda r: r["seed"])
        res = summarize(runs)
    else:
        fn = run_gpu if a.path == "gpu" else run_cpu
        if a.permutation == "randperm":  # diagnostic: SB3's uniform shuffle drawn by torch on the device
            import uav_reinforcement_learning_control_amd.ppo.ppo as ppo_mod
            ppo_mod.epoch_permutation = lambda total, device, out=None: (
                torch.randperm(total, device=device) if out is None else out.copy_(torch.randperm(total, device=device)))
        rs = []
        for s in a.seeds:
            r = fn(s, n_envs=a.n_envs, wrapper=a.wrapper)
            print(f"[{a.path} {a.wrapper} seed {s}] {r['seconds']:.1f} s  curve "
                  + " ".join(f"{v:.1f}" for v in r["curve"]), flush=True)
            rs.append(r)
        res = {"path": a.path, "wrapper": a.wrapper, "permutation": a.permutation, "n_envs": a.n_envs, "runs": rs}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
