"""PPO training driver on the MI355X env (the reference's train.py:17-146, GPU-resident).

    python -m uav_reinforcement_learning_control_amd.train --num-envs 65536 --total-timesteps 1e9
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m uav_reinforcement_learning_control_amd.train

Defaults follow train.py: HoverEnv wrapped in RateControlWrapper (:31), PPO hyperparameters
(:50-68); n_envs is the GPU batch (the reference used 16 DummyVecEnv envs on CPU). Outputs mirror
the reference's: <model-dir>/<timestamp>/config.json (the reference's fields, :88-128, read back
by evaluate.py:316-321 for the wrapper) and hover_policy_final.zip (an SB3 PPO archive, :140-141,
loadable by evaluate.py / policy_node.py's PPO.load), plus progress.csv and policy.pt.
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
    ap.add_argument("--wrapper", default="RateControlWrapper",
                    choices=["none", "RateControlWrapper", "RelPosActWrapper"])
    ap.add_argument("--num-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--total-timesteps", type=float, default=10_000_000)
    ap.add_argument("--n-steps", type=int, default=1024)
    ap.add_argument("--n-epochs", type=int, default=20)
    ap.add_argument("--n-minibatches", type=int, default=128)
    ap.add_argument("--learning-rate", type=float, default=PPOConfig.learning_rate)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log-dir", default="./logs")
    ap.add_argument("--model-dir", default="./models_trained")
    ap.add_argument("--no-graph", action="store_true", help="eager rollout (debugging)")
    return ap.parse_args(argv)


_DESCRIPTIONS = {
    "reward_function": "exp(-||pos - target||^2) of the float32 QuadState position (HoverEnv._get_reward)",
    "observation_function": "normalize([target - pos, euler(xyz), v_world, omega_body]) to [-1, 1] "
                            "(HoverEnv._get_obs)",
    "RateControlWrapper": "CTBR: rates * 360 deg/s -> PD torque (kd 26/26/18, ki 0.025, "
                          "imax 0.01) normalized by max torque",
    "RelPosActWrapper": "7-D obs [normalized rel pos (3), previous action (4)]",
}


def run_config(a, env, cfg, model, world, stamp) -> dict:
    """The reference's config.json (train.py:88-128). Its *_source / *_function fields hold
    inspect.getsource() text of the reference code; here they describe the kernel's behaviour."""
    c = env.cfg
    wname = a.wrapper if a.wrapper != "none" else "none"
    return {
        "timestamp": stamp,
        "total_timesteps": a.total_timesteps,
        "n_envs": a.num_envs * world,
        "wrapper": wname,
        "wrapper_source": _DESCRIPTIONS.get(wname),
        "reward_function": _DESCRIPTIONS["reward_function"],
        "observation_function": _DESCRIPTIONS["observation_function"],
        "observation_bounds": {"low": list(c.obs_low), "high": list(c.obs_high)},
        "state_bounds": {"low": list(c.term_low), "high": list(c.term_high)},
        "target_pos_bounds": {"low": list(c.target_low), "high": list(c.target_high)},
        "ppo": {"learning_rate": cfg.learning_rate, "n_steps": cfg.n_steps, "batch_size": model.batch,
                "n_epochs": cfg.n_epochs, "gamma": cfg.gamma, "gae_lambda": cfg.gae_lambda,
                "clip_range": cfg.clip_range, "ent_coef": cfg.ent_coef, "net_arch": list(cfg.net_arch),
                "activation_fn": "ReLU"},
        "env": a.env,
        "backend": "uav_reinforcement_learning_control_amd (MI355X kernels)",
    }


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
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    run = os.path.join(a.log_dir, stamp)
    mdir = os.path.join(a.model_dir, stamp)
    if rank == 0:
        os.makedirs(run, exist_ok=True)
        os.makedirs(mdir, exist_ok=True)
        json.dump(run_config(a, env, cfg, model, world, stamp), open(os.path.join(mdir, "config.json"), "w"),
                  indent=2)
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
        from .export import save_sb3_zip
        torch.save(model.policy.state_dict(), os.path.join(mdir, "policy.pt"))
        final = save_sb3_zip(os.path.join(mdir, "hover_policy_final"), model.policy, model.opt, cfg,
                             num_timesteps=model.num_timesteps, n_envs=a.num_envs * world,
                             batch_size=model.batch, obs_low=[-1.0] * model.obs_dim,
                             obs_high=[1.0] * model.obs_dim)
        print(f"Training complete! Model saved to {final}", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
