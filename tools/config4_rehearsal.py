#!/usr/bin/env python3
"""Config 4 rehearsal (not the measurement): 524,288 hover envs sharded over 8 ranks, PPO with one
gradient all-reduce per optimizer step -- the job `bench.py --gpus 8` runs on an 8-GPU node over RCCL
(BASELINE configs[3]; reference train_brax_ppo.py:589-620) -- run here as 8 gloo ranks that share the
one GPU of a gpurun box (RCCL refuses two ranks on one device). What it checks, at the full shape:
  * every rank's rollout shard (65,536 envs at env_id_base = rank x 65,536, 1,024 steps) is the
    same bits as the matching slice of ONE process stepping all 524,288 envs (digests of the
    advantage / reward / start-flag buffers and the last obs);
  * after the update's optimizer steps the 8 ranks hold identical parameters, and they moved.
Timings are printed but are contended (8 ranks on one GPU, gloo through the host): they are not a
scaling number. Usage: config4_rehearsal.py [world] [envs_per_rank] [n_steps] [max_minibatches]"""
import hashlib
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

DIGEST_BUFFERS = ("buf_adv", "buf_rew", "buf_start", "last_obs")


def _digest(t: torch.Tensor) -> str:
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def _shard_digests(algo, lo: int, hi: int) -> dict:
    out = {}
    for k in DIGEST_BUFFERS:
        b = getattr(algo, k)
        out[k] = _digest(b[lo:hi] if k.startswith("last") else b[:, lo:hi])
    return out


def _params(algo) -> torch.Tensor:
    return torch.cat([p.detach().reshape(-1) for p in algo.policy.parameters()])


def _rank(rank, world, port, envs, steps, mbs, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
        from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig
        env = QuadVecEnv(envs, env="hover", device="cuda:0", seed=0, env_id_base=rank * envs)
        algo = PPO(env, PPOConfig(n_steps=steps, n_epochs=20), seed=0)
        assert algo.world == world and algo._learner is not None
        p0 = _params(algo).cpu()
        rs = algo.collect_rollouts()
        dist.barrier()
        t0 = time.perf_counter()
        st = algo.train(max_minibatches=mbs)
        torch.cuda.synchronize()
        t_train = time.perf_counter() - t0
        p1 = _params(algo).cpu()
        q.put(dict(rank=rank, shard=_shard_digests(algo, 0, envs), params=_digest(p1),
                   moved=float((p1 - p0).abs().max()), n=st["n"], rollout_s=rs.seconds, train_s=t_train,
                   episodes=rs.episodes, batch=algo.batch))
        env.close()
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put(dict(rank=rank, error=repr(e)))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    envs = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    mbs = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    t0 = time.perf_counter()
    procs = [ctx.Process(target=_rank, args=(r, world, port, envs, steps, mbs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        d = q.get(timeout=900)
        res[d["rank"]] = d
        print(json.dumps(d), flush=True)
    for p in procs:
        p.join(timeout=120)
    errors = [d for d in res.values() if "error" in d]
    if errors:
        print(json.dumps({"rehearsal": "failed", "errors": errors}), flush=True)
        return 1
    t_ranks = time.perf_counter() - t0
    # the same global env ids in one process
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig
    env = QuadVecEnv(world * envs, env="hover", device="cuda:0", seed=0, env_id_base=0)
    one = PPO(env, PPOConfig(n_steps=steps, n_epochs=20), seed=0)
    one.collect_rollouts()
    shards_ok = all(_shard_digests(one, r * envs, (r + 1) * envs) == res[r]["shard"] for r in range(world))
    params_ok = len({d["params"] for d in res.values()}) == 1
    moved = min(d["moved"] for d in res.values())
    line = {"rehearsal": "config4", "world": world, "backend": "gloo (all ranks on one GPU)",
            "global_envs": world * envs, "envs_per_rank": envs, "n_steps": steps,
            "optimizer_steps": res[0]["n"], "minibatch_per_rank": res[0]["batch"],
            "shards_equal_one_process": shards_ok, "params_identical_across_ranks": params_ok,
            "params_moved": moved, "episodes_per_rank": [res[r]["episodes"] for r in range(world)],
            "contended_rollout_s": [round(res[r]["rollout_s"], 3) for r in range(world)],
            "contended_train_s": [round(res[r]["train_s"], 3) for r in range(world)],
            "ranks_wall_s": round(t_ranks, 1)}
    print(json.dumps(line), flush=True)
    env.close()
    return 0 if (shards_ok and params_ok and moved > 0) else 1


if __name__ == "__main__":
    sys.exit(main())
