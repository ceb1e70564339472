"""Brax-profile PPO training driver (the reference's train_brax_ppo.py:432-680 on the MI355X env).

    python -m uav_reinforcement_learning_control_amd.train_brax --env jax_mjx_quad --num-envs 65536

Same arguments and defaults as train_brax_ppo.py where they apply (the JAX/MJX-specific --xml,
--impl, --backend, Orbax checkpoints and --num-evals have no counterpart here). Outputs mirror the
reference's run directory: <output-dir>/<timestamp>/ppo_params.msgpack (brax model.save_params
format, ppo/brax_ppo.py + export.save_brax_params), checkpoints/params_step_<n>.msgpack every
--checkpoint-interval steps, and training_summary.json.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from datetime import datetime

import torch
import torch.distributed as dist

from .envs import QuadVecEnv
from .export import load_brax_params, save_brax_params
from .ppo.brax_ppo import BraxPPO, BraxPPOConfig


def _sizes(v: str):
    out = tuple(int(x) for x in v.split(",") if x.strip())
    if not out or any(x <= 0 for x in out):
        raise ValueError("hidden sizes must be positive integers")
    return out


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--env", default="hover", choices=["hover", "jax_mjx_quad"])
    ap.add_argument("--num-timesteps", type=int, default=2_000_000)
    ap.add_argument("--episode-length", type=int, default=500)
    ap.add_argument("--num-envs", type=int, default=1024, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--learning-rate", type=float, default=3e-4)
    ap.add_argument("--entropy-cost", type=float, default=1e-3)
    ap.add_argument("--discounting", type=float, default=0.99)
    ap.add_argument("--traj-duration-seconds", type=float, default=5.0)
    ap.add_argument("--unroll-length", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--num-minibatches", type=int, default=16)
    ap.add_argument("--num-updates-per-batch", type=int, default=4)
    ap.add_argument("--gae-lambda", type=float, default=0.95)
    ap.add_argument("--reward-scaling", type=float, default=1.0)
    ap.add_argument("--policy-hidden-sizes", default="128, 128")
    ap.add_argument("--value-hidden-sizes", default="128, 128")
    ap.add_argument("--activation", default="relu", choices=["silu", "relu", "tanh"])
    ap.add_argument("--checkpoint-interval", type=int, default=200_000)
    ap.add_argument("--restore-checkpoint-path", default=None, help="a params .msgpack to start from")
    ap.add_argument("--output-dir", default="models_brax")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = BraxPPOConfig(num_envs=a.num_envs, episode_length=a.episode_length, learning_rate=a.learning_rate,
                        entropy_cost=a.entropy_cost, discounting=a.discounting, unroll_length=a.unroll_length,
                        batch_size=a.batch_size, num_minibatches=a.num_minibatches,
                        num_updates_per_batch=a.num_updates_per_batch, gae_lambda=a.gae_lambda,
                        reward_scaling=a.reward_scaling, policy_hidden_sizes=_sizes(a.policy_hidden_sizes),
                        value_hidden_sizes=_sizes(a.value_hidden_sizes), activation=a.activation)
    kind = {"hover": "brax_hover", "jax_mjx_quad": "brax_jax_mjx"}[a.env]
    env = QuadVecEnv(a.num_envs, env=kind, device=f"cuda:{local}", seed=a.seed, env_id_base=rank * a.num_envs,
                     max_episode_steps=a.episode_length, cfg_overrides={"traj_duration": a.traj_duration_seconds})
    model = BraxPPO(env, cfg, seed=a.seed)
    if a.restore_checkpoint_path:
        norm, pol, val = load_brax_params(a.restore_checkpoint_path)
        model.net.policy.load_flax_params(pol)
        model.net.value.load_flax_params(val)
        for k in ("count", "mean", "summed_variance", "std"):
            getattr(model.norm, k).copy_(torch.as_tensor(norm[k]))
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    run = os.path.abspath(os.path.join(a.output_dir, stamp))
    ckdir = os.path.join(run, "checkpoints")
    if rank == 0:
        os.makedirs(ckdir, exist_ok=True)
    t0 = time.time()
    last_ck = 0
    stats = None
    while model.num_timesteps < a.num_timesteps:
        stats = model.training_step()
        if rank == 0:
            sps = stats.env_steps * world / stats.seconds
            print(f"step={model.num_timesteps:,} train_reward={stats.mean_episode_reward:.4f} sps={sps:.1f}",
                  flush=True)
            if a.checkpoint_interval > 0 and model.num_timesteps - last_ck >= a.checkpoint_interval:
                save_brax_params(os.path.join(ckdir, f"params_step_{model.num_timesteps}.msgpack"), model.params())
                last_ck = model.num_timesteps
    if rank == 0:
        params_path = save_brax_params(os.path.join(run, "ppo_params.msgpack"), model.params())
        summary = {"run_dir": run, "env": a.env, "num_timesteps": a.num_timesteps,
                   "episode_length": a.episode_length, "num_envs": a.num_envs * world, "seed": a.seed,
                   "learning_rate": a.learning_rate, "entropy_cost": a.entropy_cost,
                   "discounting": a.discounting, "unroll_length": a.unroll_length,
                   "batch_size": a.batch_size, "num_minibatches": a.num_minibatches,
                   "num_updates_per_batch": a.num_updates_per_batch, "gae_lambda": a.gae_lambda,
                   "reward_scaling": a.reward_scaling, "policy_hidden_sizes": list(cfg.policy_hidden_sizes),
                   "value_hidden_sizes": list(cfg.value_hidden_sizes), "activation": a.activation,
                   "traj_duration_seconds": a.traj_duration_seconds,
                   "checkpoint_interval": a.checkpoint_interval, "checkpoint_dir": ckdir,
                   "elapsed_sec": time.time() - t0,
                   "final_metrics": {"training/episode_reward": stats.mean_episode_reward if stats else None,
                                     **(stats.losses if stats else {})},
                   "params_path": params_path}
        json.dump(summary, open(os.path.join(run, "training_summary.json"), "w"), indent=2)
        print(f"Saved parameters: {params_path}", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
