"""PPO training driver on the MI355X env (the reference's train.py:17-146, GPU-resident).

    python -m uav_reinforcement_learning_control_amd.train --num-envs 65536 --total-timesteps 1e9
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m uav_reinforcement_learning_control_amd.train

Defaults follow train.py: HoverEnv wrapped in RateControlWrapper (:31), PPO hyperparameters
(:50-68); n_envs is the GPU batch (the reference used 16 DummyVecEnv envs on CPU). The run
directory gets config.json (the reference's fields, :88-128), progress.csv and the policy
state_dict with SB3 parameter names (policy.pt).
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
from .ppo import PPO, PPOConfig


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--env", default="hover", choices=["hover", "trajectory"])
    ap.add_argument("--wrapper", default="RateControlWrapper", choices=["none", "RateControlWrapper"])
    ap.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--total-timesteps", type=float, default=10_000_000)
    ap.add_argument("--n-steps", type=int, default=1024)
    ap.add_argument("--n-epochs", type=int, default=20)
    ap.add_argument("--n-minibatches", type=int, default=128)
    ap.add_argument("--learning-rate", type=float, default=PPOConfig.learning_rate)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log-dir", default="./logs")
    ap.add_argument("--no-graph", action="store_true", help="eager rollout (debugging)")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    wrapper = None if a.wrapper == "none" else a.wrapper
    env = QuadVecEnv(a.num_envs, env=a.env, wrapper=wrapper, device=f"cuda:{local}",
                     seed=a.seed, env_id_base=rank * a.num_envs)
    cfg = PPOConfig(learning_rate=a.learning_rate, n_steps=a.n_steps, n_epochs=a.n_epochs,
                    n_minibatches=a.n_minibatches)
    model = PPO(env, cfg, seed=a.seed)
    run = os.path.join(a.log_dir, datetime.now().strftime("%Y%m%d_%H%M%S"))
    if rank == 0:
        os.makedirs(run, exist_ok=True)
        json.dump({"timestamp": os.path.basename(run), "total_timesteps": a.total_timesteps,
                   "n_envs": a.num_envs * world, "wrapper": a.wrapper, "env": a.env,
                   "observation_bounds": {"low": list(env.cfg.obs_low), "high": list(env.cfg.obs_high)},
                   "state_bounds": {"low": list(env.cfg.term_low), "high": list(env.cfg.term_high)},
                   "target_pos_bounds": {"low": list(env.cfg.target_low), "high": list(env.cfg.target_high)},
                   "ppo": {**cfg.__dict__, "net_arch": list(cfg.net_arch), "activation_fn": "ReLU",
                           "batch_size": model.batch}},
                  open(os.path.join(run, "config.json"), "w"), indent=2)
        log = open(os.path.join(run, "progress.csv"), "w")
        log.write("iteration,timesteps,episodes,mean_return,mean_length,rollout_s,train_s,"
                  "rollout_env_steps_per_s,pg_loss,vf_loss,entropy,clip_fraction\n")
    it = 0
    while model.num_timesteps < a.total_timesteps:
        rs = model.collect_rollouts(use_graph=not a.no_graph)
        t0 = time.perf_counter()
        ts = model.train()
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        it += 1
        if rank == 0:
            fps = rs.env_steps * world / rs.seconds
            line = (f"{it},{model.num_timesteps},{rs.episodes},{rs.mean_return:.4f},{rs.mean_length:.2f},"
                    f"{rs.seconds:.3f},{tt:.3f},{fps:.4g},{ts['pg_loss']:.5f},{ts['vf_loss']:.5f},"
                    f"{ts['entropy']:.4f},{ts['clip_fraction']:.4f}")
            log.write(line + "\n"); log.flush()
            print(line, flush=True)
    if rank == 0:
        torch.save(model.policy.state_dict(), os.path.join(run, "policy.pt"))
        print(f"saved {run}/policy.pt", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
