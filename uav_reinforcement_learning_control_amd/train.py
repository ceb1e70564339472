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
    # the reference's callbacks (train.py:71-86)
    ap.add_argument("--checkpoint-freq", type=float, default=50_000,
                    help="CheckpointCallback: save hover_policy_<steps>_steps.zip (+ a resumable .pt) "
                         "every this many timesteps (checked after each PPO iteration; 0 = off)")
    ap.add_argument("--eval-freq", type=float, default=10_000,
                    help="EvalCallback: evaluate every this many timesteps (0 = off)")
    ap.add_argument("--n-eval-episodes", type=int, default=5)
    ap.add_argument("--resume", default=None,
                    help="resume from a checkpoint .pt (policy, optimizer, timesteps, noise counter)")
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


def _save_zip(path, model, cfg, n_envs):
    from .export import save_sb3_zip
    return save_sb3_zip(path, model.policy, model.opt, cfg, num_timesteps=model.num_timesteps, n_envs=n_envs,
                        batch_size=model.batch, obs_low=[-1.0] * model.obs_dim, obs_high=[1.0] * model.obs_dim)


class Checkpointer:
    """SB3 CheckpointCallback(save_freq, save_path=model_dir, name_prefix="hover_policy")
    (train.py:71-75): hover_policy_<num_timesteps>_steps.zip each time another `freq` timesteps
    have passed, plus the same name with .pt holding what --resume needs (PPO.state_dict())."""

    def __init__(self, model_dir, freq, model, cfg, n_envs):
        self.dir, self.freq, self.model, self.cfg, self.n_envs = model_dir, float(freq), model, cfg, n_envs
        self.next = model.num_timesteps + self.freq

    def step(self):
        if self.freq <= 0 or self.model.num_timesteps < self.next:
            return None
        while self.next <= self.model.num_timesteps:
            self.next += self.freq
        base = os.path.join(self.dir, f"hover_policy_{self.model.num_timesteps}_steps")
        _save_zip(base, self.model, self.cfg, self.n_envs)
        torch.save(self.model.state_dict(), base + ".pt")
        return base


class EvalCallback:
    """SB3 EvalCallback(eval_env, best_model_save_path=model_dir, log_path=log_dir, eval_freq,
    n_eval_episodes=5, deterministic=True) (train.py:78-86): every `freq` timesteps, run
    n_eval_episodes fresh episodes of the training env kind with the deterministic policy (all
    at once on the GPU, evaluate.evaluate_episodes); append to <log_dir>/evaluations.npz
    (timesteps, results, ep_lengths) and save best_model.zip when the mean reward improves."""

    def __init__(self, log_dir, model_dir, freq, n_episodes, wrapper, env_kind, model, cfg, n_envs, device, seed):
        self.log_dir, self.model_dir, self.freq, self.n = log_dir, model_dir, float(freq), int(n_episodes)
        self.wrapper, self.env_kind, self.model, self.cfg, self.n_envs = wrapper, env_kind, model, cfg, n_envs
        self.device, self.seed = device, seed
        self.next = model.num_timesteps + self.freq
        self.best = -float("inf")
        self.timesteps, self.results, self.lengths = [], [], []

    def step(self):
        if self.freq <= 0 or self.model.num_timesteps < self.next:
            return None
        while self.next <= self.model.num_timesteps:
            self.next += self.freq
        from .evaluate import evaluate_episodes
        r = evaluate_episodes(self.model.policy, num_episodes=self.n, wrapper=self.wrapper, env=self.env_kind,
                              device=self.device, seed=self.seed + 7919 * (len(self.timesteps) + 1))
        self.timesteps.append(self.model.num_timesteps)
        self.results.append(r["rewards"])
        self.lengths.append(r["lengths"])
        import numpy as np
        np.savez(os.path.join(self.log_dir, "evaluations.npz"), timesteps=np.array(self.timesteps),
                 results=np.array(self.results), ep_lengths=np.array(self.lengths))
        print(f"Eval num_timesteps={self.model.num_timesteps}, episode_reward={r['mean_reward']:.2f} "
              f"+/- {r['std_reward']:.2f}, episode_length={r['mean_length']:.2f}", flush=True)
        if r["mean_reward"] > self.best:
            self.best = r["mean_reward"]
            _save_zip(os.path.join(self.model_dir, "best_model"), self.model, self.cfg, self.n_envs)
            print("New best mean reward!", flush=True)
        return r


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
    if a.resume:
        model.load_state_dict(torch.load(a.resume, map_location=env.device, weights_only=True))
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
    ckpt = Checkpointer(mdir, a.checkpoint_freq, model, cfg, a.num_envs * world) if rank == 0 else None
    evalcb = (EvalCallback(run, mdir, a.eval_freq, a.n_eval_episodes, wrapper, a.env, model, cfg,
                           a.num_envs * world, env.device, a.seed) if rank == 0 else None)
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
            ckpt.step()
            evalcb.step()
    if rank == 0:
        torch.save(model.policy.state_dict(), os.path.join(mdir, "policy.pt"))
        torch.save(model.state_dict(), os.path.join(mdir, "hover_policy_final.pt"))
        final = _save_zip(os.path.join(mdir, "hover_policy_final"), model, cfg, a.num_envs * world)
        print(f"Training complete! Model saved to {final}", flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
