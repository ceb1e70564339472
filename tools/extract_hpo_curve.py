"""Extract the reference's learning-level anchor for row P into a committed fixture.

The reference's Optuna study (``/root/reference/optuna_full.db``, study ``ppo_hover``) holds, for
trial 31 -- the trial whose parameters ``train.py:50-68`` hard-codes -- the mean reward of each of
its 10 ``TrialEvalCallback`` evaluations (``optimize.py:85-117``): 10 deterministic episodes over 5
eval envs (``optimize.py:266-270``) every ``n_timesteps // 10`` = 50,000 env steps
(``optimize.py:244,254``) of a 500,000-step, 8-env run (``optimize.py:244-245``).

Run only where ``/root/reference`` exists (the build container). The database is opened read-only
with sqlite3; optuna itself is not needed (and is absent). Writes ``tests/golden/hpo_trial31.json``.
"""
from __future__ import annotations

import json
import os
import sqlite3
import sys

DB = "/root/reference/optuna_full.db"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "hpo_trial31.json")
TRIAL = 31


def categorical(value: float, dist: str):
    """Optuna stores a categorical parameter as the index of its choice."""
    d = json.loads(dist)
    if d["name"] == "CategoricalDistribution":
        return d["attributes"]["choices"][int(value)]
    return value


def main() -> int:
    if not os.path.exists(DB):
        print(f"{DB} not found: run in the build container", file=sys.stderr)
        return 1
    con = sqlite3.connect(f"file:{DB}?mode=ro", uri=True)
    cur = con.cursor()
    (study,) = cur.execute("select study_name from studies").fetchone()
    tid, state, t0, t1 = cur.execute(
        "select trial_id, state, datetime_start, datetime_complete from trials where number = ?", (TRIAL,)).fetchone()
    params = {name: categorical(v, dist) for name, v, dist in
              cur.execute("select param_name, param_value, distribution_json from trial_params where trial_id = ?",
                          (tid,))}
    attrs = {k: json.loads(v) for k, v in
             cur.execute("select key, value_json from trial_user_attributes where trial_id = ?", (tid,))}
    (final,) = cur.execute("select value from trial_values where trial_id = ?", (tid,)).fetchone()
    curve = [v for _, v in cur.execute(
        "select step, intermediate_value from trial_intermediate_values where trial_id = ? order by step", (tid,))]
    n_timesteps, n_envs, n_eval = 500_000, 8, 10
    out = {
        "source": f"{DB} (study '{study}', trial {TRIAL}, {state}, {t0} .. {t1}); tools/extract_hpo_curve.py",
        "params": params,
        "user_attrs": attrs,
        "final_value": final,
        "eval_timesteps": [n_timesteps // n_eval * (k + 1) for k in range(n_eval)],
        "eval_mean_reward": curve,
        "run": {
            "n_timesteps": n_timesteps, "n_envs": n_envs, "n_eval_envs": 5, "n_eval_episodes": 10,
            "eval_freq_env_steps": n_timesteps // n_eval, "deterministic_eval": True,
            "wrapper": "RateControlWrapper", "net_arch": [128, 128], "activation_fn": "ReLU",
            "cites": ["optimize.py:26 (wrapper_cls)", "optimize.py:33-74 (search space)",
                      "optimize.py:127-180 (batch clamp, make_vec_env, EvalCallback)",
                      "optimize.py:244-245 (500k steps, 8 envs)", "optimize.py:254 (eval_freq)",
                      "optimize.py:266-270 (5 eval envs, 10 episodes)", "train.py:50-68 (same params)"],
        },
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {os.path.normpath(OUT)}: final {final:.2f}, curve {[round(v, 1) for v in curve]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
