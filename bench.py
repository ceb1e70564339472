#!/usr/bin/env python3
"""Throughput of the MI355X-native HoverEnv step (the reference's hot path), env-steps/s.

Workload (BASELINE.json metric): 65,536 HoverEnv envs per GPU, one process per GPU, global env
ids contiguous per rank (a shard is bit-identical to the same ids on one GPU). One bench "step"
= one fused quad_step launch over the rank's batch: CTBR-off HoverEnv.step (mixer, voltage sag,
MuJoCo-equivalent physics, obs, reward, termination, truncation) + SB3 auto-reset, actions
U[-1,1)^4 pre-generated in HBM (action_space.sample(), debug_training.py:111 / configs[1]).
The timed loop replays hipGraphs of the step launches (launch-bound at this size).

Prints ONE JSON line (rank 0). Also measured in the same run and reported as extra keys:
per-launch kernel time from HIP event pairs (-> roofline), the 1M-env HBM-bound point, and the
CPU baseline (the float64 oracle, 1 core, bounded sample) -- see DESIGN.md "Measurement".
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec (whole node) at 65 536 hover envs, 1/2/4/8 MI355X"
ENVS_PER_GPU = 65536
BYTES_PER_ENV_STEP = 278  # state r/w 2x104, action 16, obs+rew+term+trunc 54
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _quad_step_fn(env):
    """Pre-built direct C-ABI call (no Python-side tensor ops per step)."""
    from uav_reinforcement_learning_control_amd import _native as N
    L = N.lib()
    out = N.QuadStepOut(obs=env.obs.data_ptr(), reward=env.reward.data_ptr(),
                        terminated=env.terminated.data_ptr(), truncated=env.truncated.data_ptr(),
                        terminal_obs=env.terminal_obs.data_ptr())
    h = env._h

    def step(actions_ptr: int):
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        rc = L.quad_step(h, C.c_void_p(actions_ptr), C.byref(out), s)
        if rc != 0:
            N.check(rc, "quad_step")
    return step


def _graph_of(step, actions, first: int, n: int):
    """Capture n step launches (action batches first.. in order) into one hipGraph and upload its
    executable, so that its first replay does not pay instantiation/upload costs."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(n):
            step(actions[(first + k) % len(actions)].data_ptr())
    _graph_upload(g)
    return g


def _graph_upload(g) -> None:
    """hipGraphUpload of a captured torch graph's executable on the current stream (torch already
    loaded the HIP runtime, so dlopen by soname returns that same library)."""
    try:
        hip = C.CDLL("libamdhip64.so.7")
        rc = hip.hipGraphUpload(C.c_void_p(g.raw_cuda_graph_exec()),
                                C.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipGraphUpload returned {rc}")
    except (AttributeError, OSError):
        pass  # older torch without raw_cuda_graph_exec: the untimed warm replay below covers it


def _gated_kernel_us(step, actions, n_launch: int = 200) -> float:
    """Average device time per launch of back-to-back graph-replayed step launches, HIP events on
    the launching stream. A short spin kernel ahead of the first event keeps the GPU busy while
    the host submits, so the interval holds only the launches (the roofline's kernel time)."""
    chunk = 100
    g = _graph_of(step, actions, 0, chunk)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(200_000)  # ~100 us gate
    e0.record()
    for _ in range(max(1, n_launch // chunk)):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (max(1, n_launch // chunk) * chunk)


def _launch_floor_us(n_launch: int = 400) -> float:
    """Device time per launch of an (almost) empty kernel graph-replayed back to back on the
    current stream, timed like _gated_kernel_us: the dispatch floor every one-launch step pays
    whatever it does (1.61-1.63 us on MI355X for any grid from 64 x 128 to 2048 x 64 threads,
    tools/diag/launch_floor.hip, profiles/r04/r4_launch_floor.txt)."""
    chunk = 100
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(chunk):
            torch.cuda._sleep(0)
    _graph_upload(g)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(200_000)
    e0.record()
    for _ in range(max(1, n_launch // chunk)):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (max(1, n_launch // chunk) * chunk)


def _kernel_name(env) -> str:
    """The step kernel form the handle actually launches (quad_kernel_form: 16 SPEC | 32 helper waves |
    128 256-env blocks | 256 nt | 512 k_step_hd)."""
    from uav_reinforcement_learning_control_amd import _native as N
    form = int(N.lib().quad_kernel_form(env._h))
    name = ("k_step_hd" if form & 512 else "k_step_h") + "<HOVER,noCTBR>"
    tags = (["SPEC constants"] if form & 16 else []) + (["helper waves draw the resets"] if form & 32 else []) + \
        (["nt state loads/stores"] if form & 256 else []) + (["7-wave DRAM form k_step_hd"] if form & 512 else [])
    return name + (f" ({', '.join(tags)})" if tags else "")


def _kernel_symbol(env) -> str:
    """The launched hover step kernel's template symbol as rocprofv3 names it (csrc/quadenv.hip
    quad_step_range: k_step_h<KIND, CTBR, SPEC, HB, NT> with HB from quad_kernel_form bit 7 (256-env
    blocks for 32,769 .. 2,097,151 envs, else 64) and NT (the state's nt cache policy) from bit 8;
    k_step_hd<KIND, CTBR, SPEC> when bit 9 is set)."""
    from uav_reinforcement_learning_control_amd import _native as N
    form = int(N.lib().quad_kernel_form(env._h))
    spec = "true" if form & 16 else "false"
    if form & 512:
        return f"k_step_hd<0, false, {spec}>"
    return f"k_step_h<0, false, {spec}, {256 if form & 128 else 64}, {'true' if form & 256 else 'false'}>"


def _run_rank(args, rank, world, local_rank):
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv

    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    n = args.envs
    env = QuadVecEnv(n, env="hover", device=dev, seed=args.seed, env_id_base=rank * n)
    env.reset()
    n_act = min(args.action_batches, args.steps + args.warmup)
    actions = [env.random_actions(k) for k in range(n_act)]  # resident in HBM
    step = _quad_step_fn(env)
    chunk = args.graph_chunk if args.steps % args.graph_chunk == 0 else args.steps

    def region(graphs):
        """barrier + synchronize, the replays between two HIP events (on the stream the kernels
        run on: the device time of the same region), synchronize; returns (wall s, e0, e1)"""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for gr in graphs:
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, e0, e1

    # the timed step sequence as hipGraph(s), captured and uploaded before the warmup; the W
    # warmup steps are replays of a graph of the same launches (first kernel runs, caches, TLB),
    # run through the timed region's own host path: its first execution in a process costs ~10 us
    # of host time (event records, synchronize; profiles/r02/first_region.txt), setup, not steps
    g = _graph_of(step, actions, args.warmup, chunk)
    if args.warmup > 0:
        gw = _graph_of(step, actions, 0, args.warmup)
        region([gw])

    # timed region: exactly K steps, barrier + synchronize on both sides
    elapsed, e0, e1 = region([g] * (args.steps // chunk))
    # the closing barrier follows this rank's clock stop: its RCCL latency (tens of us against a
    # ~130 us 20-step region) is not step work; the MAX over ranks below is the slowest rank's K steps
    if world > 1:
        dist.barrier()
    region_us = e0.elapsed_time(e1) * 1e3 / args.steps
    own_elapsed = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-launch kernel time (roofline) on the same kernel, stream and data
    res = dict(elapsed=elapsed, region_us=region_us,
               kernel_us=_gated_kernel_us(step, actions, args.kernel_launches),
               kernel=_kernel_name(env), symbol=_kernel_symbol(env), launch_floor_us=_launch_floor_us())
    if world > 1:  # every rank's own figures: a slow GPU or link shows here, not only in the MAX
        res["per_rank"] = _per_rank(dict(elapsed_s=own_elapsed, region_us=region_us, kernel_us=res["kernel_us"]),
                                    ("elapsed_s", "region_us", "kernel_us"))
    if args.rollout_steps > 0:
        res["rollout"] = _rollout_phase(env, args)
    if args.e2e_iters > 0:
        res["end_to_end"] = _end_to_end(env, args, world)
        if world > 1:
            res["end_to_end"]["shard_identity"] = _shard_identity(args, rank, world, dev)
    if rank == 0 and not args.no_configs:
        res["configs"] = {
            "config2_hover_4096": _kernel_rate(4096, "hover", None, dev, args.seed),
            "config2_hover_4096_one_launch": _kstep_rate(4096, 1000, dev, args.seed),
            "hover_65536_one_launch_random": _kstep_rate(65536, 200, dev, args.seed),
            "config5_traj_ctbr_65536": _kernel_rate(65536, "trajectory", "RateControlWrapper", dev, args.seed),
            "hover_ctbr_65536": _kernel_rate(65536, "hover", "RateControlWrapper", dev, args.seed)}
        if world == 1:  # a one-process PPO (at world > 1 its construction would join the ranks' collectives)
            res["configs"]["config1_train_py_on_gpu"] = _train_py_scale(dev, args.seed)
    del actions, g
    env.close()
    if rank == 0:
        torch.cuda.empty_cache()
        if args.large_envs > 0:  # Infinity-Cache-assisted (~290 MB working set)
            res["large"] = _large_point(args.large_envs, dev, args.seed, 200)
        if args.dram_envs > 0:  # true HBM: 1.2 GB per launch, 4.5x the 256 MB Infinity Cache
            res["dram"] = _large_point(args.dram_envs, dev, args.seed, 40)
    return res


def _mem_floor_fn(env):
    """quad_mem_floor on the env's own tiles and output rows: the step's 278 B per env with no
    compute, quad_step's cache policy for this size (the same-run memory floor of the step)."""
    from uav_reinforcement_learning_control_amd import _native as N
    L = N.lib()
    out = N.QuadStepOut(obs=env.obs.data_ptr(), reward=env.reward.data_ptr(),
                        terminated=env.terminated.data_ptr(), truncated=env.truncated.data_ptr())
    h = env._h

    def floor(actions_ptr: int):
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        rc = L.quad_mem_floor(h, C.c_void_p(actions_ptr), C.byref(out), s)
        if rc != 0:
            N.check(rc, "quad_mem_floor")
    return floor


def _per_rank(mine: dict, keys) -> dict:
    """Gather one dict of figures from every rank (all_gather_object, a collective: every rank calls
    it); for each key in `keys` the per-rank list with min / max / argmax rank and max / min."""
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, dict(mine, rank=dist.get_rank()))
    out = {"ranks": got}
    for k in keys:
        v = [g[k] for g in got]
        if any(x is None for x in v):
            continue
        hi = max(range(len(v)), key=v.__getitem__)
        out[k] = {"min": min(v), "max": v[hi], "argmax_rank": hi, "max_over_min": v[hi] / min(v) if min(v) > 0 else None}
    return out


def _large_point(n, dev, seed, launches) -> dict:
    """The same step at a large batch (the size's default kernel form) after 50 steps (the
    post-reset transient: ~11 % of envs reset per step from there on): gated per-launch time,
    HBM roofline of the algorithmic bytes, and the committed PMC traffic of that kernel and size.
    Beside it, in the same process on the same buffers, the copy floor: quad_mem_floor's
    per-launch time (the same loads and stores, no compute), timed the same way before and after
    the step (their mean), so the step's distance from what this box's HBM delivers for its access
    pattern is separated from the box-to-box spread of the absolute figure."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    big = QuadVecEnv(n, env="hover", device=dev, seed=seed)
    big.reset()
    acts = [big.random_actions(k) for k in range(8)]
    st = _quad_step_fn(big)
    for k in range(50):
        st(acts[k % 8].data_ptr())
    fl = _mem_floor_fn(big)
    floor0 = _gated_kernel_us(fl, acts, launches)
    us = _gated_kernel_us(st, acts, launches)
    floor1 = _gated_kernel_us(fl, acts, launches)
    floor_us = 0.5 * (floor0 + floor1)
    sym = _kernel_symbol(big)
    big.close()
    del acts
    torch.cuda.empty_cache()
    gbs = BYTES_PER_ENV_STEP * n / (us * 1e-6) / 1e9
    return {"envs": n, "kernel_us": us, "env_steps_per_s_kernel": n / (us * 1e-6), "achieved_GBs": gbs,
            "frac": gbs / HBM_PEAK_GBS, "copy_floor_us": floor_us, "copy_floor_us_before_after": [floor0, floor1],
            "copy_floor_GBs": BYTES_PER_ENV_STEP * n / (floor_us * 1e-6) / 1e9,
            "frac_of_copy_floor": floor_us / us,
            "copy_floor_what": "quad_mem_floor: the step's 278 B/env of loads and stores on the same tiles "
                               "and rows with quad_step's cache policy, no compute (same process, same buffers)",
            "kernel_symbol": sym, "traffic_pmc": _pmc_traffic(sym, n), "issue": _pmc_issue(sym, n)}


def _kernel_rate(n, kind, wrapper, dev, seed) -> dict:
    """Env-step kernel time for another SURVEY 8(d) config (graph of 20 launches, 10 replays)."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    e = QuadVecEnv(n, env=kind, wrapper=wrapper, device=dev, seed=seed)
    e.reset()
    acts = [e.random_actions(k) for k in range(4)]
    st = _quad_step_fn(e)
    for k in range(50):
        st(acts[k % 4].data_ptr())
    us = _gated_kernel_us(st, acts, 200)
    e.close()
    bpe = BYTES_PER_ENV_STEP + (24 if wrapper else 0)
    return {"envs": n, "env": kind, "wrapper": wrapper, "kernel_us": us,
            "env_steps_per_s": n / (us * 1e-6), "achieved_GBs": bpe * n / (us * 1e-6) / 1e9}


def _train_py_scale(dev, seed, iters: int = 2) -> dict:
    """SURVEY config 1's workload -- train.py's PPO iteration (16 HoverEnv + RateControlWrapper envs x
    1,024 steps, then 20 epochs x 128 minibatches of 128 rows = 2,560 Adam steps) -- on the GPU path
    (quad_rollout, quad_ppo_grad, quad_clip_adam; each epoch's optimizer steps one hipGraph replay),
    beside cpu_baseline_ppo's CPU timing of the same iteration. One untimed iteration first."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig
    env = QuadVecEnv(16, env="hover", wrapper="RateControlWrapper", device=dev, seed=seed)
    m = PPO(env, PPOConfig(batch_size=128), seed=0)
    m.collect_rollouts()
    m.train()
    torch.cuda.synchronize()
    t_roll = t_train = 0.0
    for _ in range(iters):
        t0 = time.perf_counter()
        rs = m.collect_rollouts()
        t1 = time.perf_counter()
        m.train()
        torch.cuda.synchronize()
        t_roll += t1 - t0
        t_train += time.perf_counter() - t1
    steps = rs.env_steps
    opt_steps = m.cfg.n_epochs * m.n_minibatches_per_epoch()
    out = {"envs": 16, "n_steps": m.cfg.n_steps, "batch_size": m.batch, "optimizer_steps": opt_steps,
           "rollout_s": t_roll / iters, "train_s": t_train / iters,
           "us_per_optimizer_step": 1e6 * t_train / iters / opt_steps,
           "env_steps_per_s": steps * iters / (t_roll + t_train), "graph_update": m._epoch_graph is not None}
    del m
    env.close()
    return out


def _kstep_rate(n, steps, dev, seed) -> dict:
    """SURVEY config 2 as one launch (quad_step_random): `steps` random-action steps with state kept
    on chip, actions drawn in-kernel from quad_random_actions' map; HIP events on the launch's
    stream after one untimed launch. Per step the same outputs go to HBM as with quad_step."""
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    e = QuadVecEnv(n, env="hover", device=dev, seed=seed)
    e.reset()
    e.step_random(50, step0=0)  # warm-up (not timed)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = e.step_random(steps, step0=50)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / steps
    resets = float((r["terminated"] | r["truncated"]).float().mean())
    del r
    e.close()
    return {"envs": n, "steps_per_launch": steps,
            "kernel": "k_step_random_h<HOVER,noCTBR> (helper waves draw actions and resets)",
            "us_per_step": us, "env_steps_per_s": n / (us * 1e-6), "reset_fraction_per_step": resets,
            "bytes_per_env_step_out": 70, "note": "state read/written once per launch; actions drawn in-kernel"}


def _end_to_end(env, args, world: int = 1) -> dict:
    """One full PPO iteration per SURVEY 8(d) config 3: rollout of n_steps (MFMA policy path) +
    GAE + the SB3-schedule update (n_epochs x n_minibatches Adam steps on the rollout buffer).
    At world > 1 (config 4) also: the ranks as torch.distributed sees them, every gradient
    all-reduce of the timed update HIP-event timed (allreduce_mean_) with its share of the optimizer
    step, the same collective alone, and the episode statistics reduced over the ranks."""
    from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig
    cfg = PPOConfig(n_steps=args.e2e_steps, n_epochs=args.e2e_epochs)
    m = PPO(env, cfg, seed=0)
    first = m.collect_rollouts(use_graph=True)  # capture + warm (not timed)
    first_stats = m._done_stats.tolist()  # the whole job's (reduced over ranks), before any update
    # warm-up (not timed): on one GPU two epochs capture the update's per-epoch hipGraph (PPO.
    # _train_graphed; setup, like the rollout's graph capture above); otherwise two minibatches
    m.train(n_epochs=2) if world == 1 and m._learner is not None else m.train(n_epochs=1, max_minibatches=2)
    torch.cuda.synchronize()
    t_roll = t_train = 0.0
    if world > 1:
        m.comm_events = []  # time every gradient all-reduce of the timed updates
    for _ in range(args.e2e_iters):
        rs = m.collect_rollouts(use_graph=True)
        t0 = time.perf_counter()
        m.train()
        torch.cuda.synchronize()
        t_train += time.perf_counter() - t0
        t_roll += rs.seconds
    comm = m.comm_stats() if world > 1 else None
    steps = args.e2e_iters * rs.env_steps * world  # every rank's envs (config 4 at N = 8)
    wall = t_roll + t_train
    per_rank = None
    if world > 1:  # every rank's iteration and all-reduce figures (skew), then the slowest rank
        per_rank = _per_rank(dict(wall_s=wall, rollout_s=t_roll / args.e2e_iters, train_s=t_train / args.e2e_iters,
                                  allreduce_median_us=comm["median_us"] if comm else None,
                                  allreduce_mean_us=comm["mean_us"] if comm else None,
                                  allreduce_max_us=comm["max_us"] if comm else None),
                             ("wall_s", "train_s", "allreduce_median_us", "allreduce_max_us"))
    if world > 1:  # the slowest rank sets the whole job's time
        t = torch.tensor([wall], dtype=torch.float64, device=env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    opt_steps = max(1, cfg.n_epochs * m.n_minibatches_per_epoch())
    ms_opt = 1e3 * t_train / args.e2e_iters / opt_steps
    out = {"world_size": world, "n_ranks": dist.get_world_size() if world > 1 else 1,
           "global_envs": env.num_envs * world,
           "grad_allreduce": "one flat fp32 bucket (37,001 params) per optimizer step" if world > 1 else None,
           "n_steps": cfg.n_steps, "n_epochs": cfg.n_epochs, "minibatches_per_epoch": m.n_minibatches_per_epoch(),
           "minibatch": m.batch, "iterations": args.e2e_iters,
           "rollout_s": t_roll / args.e2e_iters, "train_s": t_train / args.e2e_iters,
           "update_path": "quad_ppo_grad (fused fwd+loss+bwd on MFMA) + quad_clip_adam"
           if m._learner is not None else "torch autograd",
           "ms_per_optimizer_step": ms_opt,
           "env_steps_per_s": steps / wall,
           "episodes_first_rollout": {"return_sum": first_stats[0], "length_sum": first_stats[1],
                                      "count": int(first_stats[2]), "local_count": first.extra["local_episodes"],
                                      "reduced_over_ranks": world > 1}}
    if per_rank is not None:
        out["per_rank"] = per_rank
    if world > 1:
        alone = _allreduce_alone(m)
        out["allreduce"] = dict(
            comm, what="HIP events on the optimizer step's stream around dist.all_reduce(SUM) of the "
                       "148 KB bucket and work.wait() (ppo.allreduce_mean_), every optimizer step of the "
                       "timed update(s)",
            backend=dist.get_backend(), exposed_share_of_optimizer_step=comm["mean_us"] / (ms_opt * 1e3),
            alone=alone)
    if m._learner is not None:
        out["learner_kernel"] = _learner_kernel(m)
    del m
    torch.cuda.empty_cache()
    return out


def _allreduce_alone(m, reps: int = 50) -> dict:
    """The gradient bucket's all-reduce by itself (no update around it): `reps` back-to-back
    SUM all-reduces of a copy of the 148 KB bucket, HIP-event timed on the current stream."""
    buf = m._flat.clone()
    for _ in range(5):
        dist.all_reduce(buf)
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dist.all_reduce(buf)
    e1.record()
    torch.cuda.synchronize()
    return {"reps": reps, "us_per_allreduce": e0.elapsed_time(e1) * 1e3 / reps, "bytes": buf.numel() * 4}


def _shard_identity(args, rank: int, world: int, dev, steps: int = 16) -> dict:
    """Config 4's sharding check: rank r steps envs [r N, (r + 1) N) of the global
    batch from a fresh handle (reset, then `steps` steps of the global-id-keyed random actions,
    SB3 auto-reset on); its SHA-256 digest of every obs / reward / flag / terminal-obs output must
    equal the digest rank 0 forms from the same rows of ONE handle of all world x N envs."""
    import hashlib
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    n = args.envs

    def run(e, lo, hi):
        hs = [hashlib.sha256() for _ in range(lo, hi, n)]

        def add(outs):
            for j, a in enumerate(range(lo, hi, n)):
                for t in outs:
                    hs[j].update(t[a - lo:a - lo + n].contiguous().cpu().numpy().tobytes())
        add([e.reset()])
        for k in range(steps):
            obs, rew, te, tr, inf = e.step(e.random_actions(k))
            add([obs, rew, te, tr, inf["terminal_observation"]])
        return [h.hexdigest() for h in hs]

    mine = QuadVecEnv(n, env="hover", device=dev, seed=args.seed, env_id_base=rank * n)
    d = run(mine, 0, n)[0]
    mine.close()
    got = [None] * world
    dist.all_gather_object(got, d)
    if rank != 0:
        return {}
    one = QuadVecEnv(world * n, env="hover", device=dev, seed=args.seed, env_id_base=0)
    ref = run(one, 0, world * n)
    one.close()
    torch.cuda.empty_cache()
    return {"steps": steps, "envs_per_rank": n, "one_handle_envs": world * n,
            "rank_digests": [g[:16] for g in got], "one_handle_digests": [r[:16] for r in ref],
            "all_equal": all(g == r for g, r in zip(got, ref))}


def _learner_kernel(m) -> dict:
    """quad_ppo_grad alone on the rollout buffer, over consecutive minibatches of the training's own
    epoch permutation (ppo.epoch_permutation -> quad_permutation, as PPO.train draws them),
    HIP-event timed on its stream: the MFMA roofline of the update. Also the whole fused optimizer
    step (quad_ppo_grad + quad_clip_adam) over the same minibatches, to set beside the end-to-end
    ms_per_optimizer_step (which adds the host loop). FLOP = the issued products per row."""
    from uav_reinforcement_learning_control_amd.ppo.ppo import epoch_permutation
    total = m.buf_obs.shape[0] * m.buf_obs.shape[1]
    obs, act = m.buf_obs.view(total, -1), m.buf_act.view(total, 4)
    lp, adv, ret = m.buf_logp.view(total), m.buf_adv.view(total), m.buf_ret.view(total)
    perm = epoch_permutation(total, obs.device)
    B = m.batch
    nmb = max(1, total // B)
    reps = min(20, nmb)
    idx = [perm[k * B:(k + 1) * B] for k in range(reps)]
    m._learner.grads(obs, act, lp, adv, ret, idx[0])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(reps):
        m._learner.grads(obs, act, lp, adv, ret, idx[k])
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    saved = [p.detach().clone() for p in m.params]  # (the optimizer steps below are undone)
    saved_opt = {k: {n: (t.clone() if torch.is_tensor(t) else t) for n, t in v.items()} for k, v in m.opt.state.items()}
    e0.record()
    for k in range(reps):
        m._learner.grads(obs, act, lp, adv, ret, idx[k])
        m._adam.step()
    e1.record()
    torch.cuda.synchronize()
    us_step = e0.elapsed_time(e1) * 1e3 / reps
    with torch.no_grad():
        for p, q in zip(m.params, saved):
            p.copy_(q)
    for k, v in saved_opt.items():
        m.opt.state[k].update(v)
    # the f32 algorithm's MFMA work per row per net: (12 + 128 + 128 + 128 + 32) 32x32x2 per 64 rows
    # per wave x 4 waves, plus 32 16x16x4 (half the cycles) -> 444 x 2048 x 2 flop x 4 / 64 rows
    flop = 2 * B * (444 * 2048 * 2 * 4 / 64)
    from uav_reinforcement_learning_control_amd import _native as N
    form = int(N.lib().quad_ppo_grad_form())
    out = {"kernel": "quad_ppo_grad (%s + k_ppo_reduce)" % ("k_x3_prep + k_ppo_grad_x3" if form else "k_adv_stats + k_ppo_grad"),
           "rows": B, "index_source": "epoch_permutation (quad_permutation), consecutive minibatches",
           "us_per_minibatch": us, "us_per_optimizer_step_device": us_step, "issued_flop": flop}
    if form:
        # bf16x3: per 64-row round and wave 324 v_mfma_f32_32x32x16_bf16 (32 cycles each: L1 12, L2 96,
        # dW2 96, dh1 96, dW1 24); db2 and dW3 are per-lane VALU sums since round 3 (until then 12 more
        # bf16 MFMAs and 32 f32 16x16x4 per round, which this floor counted)
        cyc = 2 * (B / 64) * 4 * (324 * 32) / 1024  # per SIMD, both nets
        floor_us = cyc / 2.4e3  # at the 2.4 GHz peak clock
        out.update({"roofline": {"bound": "mfma", "unit": "matrix-pipe time", "floor_us": floor_us,
                                 "frac": floor_us / us,
                                 "what": "324 v_mfma_f32_32x32x16_bf16 (32 cycles each) per 64-row round "
                                         "and wave, both nets, 1,024 SIMDs at 2.4 GHz"},
                    "matrix_pipe_floor_us": floor_us, "matrix_pipe_frac": floor_us / us,
                    "derived_f32_equivalent_TFLOPs": flop / us / 1e6})
    else:
        out.update({"achieved_TFLOPs": flop / us / 1e6, "peak_TFLOPs": 157.3, "bound": "mfma (fp32 32x32x2)"})
    return out


def _rollout_phase(env, args) -> dict:
    """PPO rollout phase on the same 65,536 envs, timed over n_steps, GAE included, three ways:
    the one-launch rollout (quad_rollout: policy + env step + bootstrap + statistics for all steps
    in one kernel, the PPO default), the two-launch MFMA path (policy kernel + env step per step,
    graph-replayed) and the same step as torch ops on the same policy."""
    from uav_reinforcement_learning_control_amd.ppo import PPO, PPOConfig
    out = {"n_steps": args.rollout_steps,
           "what": "actor+critic MLP 12-128-128 (f32-level, bf16x3 MFMA) + Gaussian sample + clip + env step + "
                   "TimeLimit bootstrap + buffer rows; GAE included"}
    n = env.num_envs
    flop_step = n * (2 * 2 * (12 * 128 + 128 * 128) + 2 * 128 * 5)  # both nets + heads, per env-step

    def mlp_roofline(flop, us, steps):
        # bf16 MFMA on three-piece splits (csrc/policy_net.h): per 64 envs (one wave, two 32-env
        # tiles) and step, (4 layer-1 + 32 layer-2) k-steps x 6 v_mfma_f32_32x32x16_bf16 x 2 tiles
        # x 2 nets = 864 MFMAs of 32 cycles on the wave's SIMD
        floor_us = steps * 864 * 32 * (n / 64) / 1024 / 2.4e3  # 1,024 SIMDs at the 2.4 GHz peak clock
        # the roofline is the matrix pipe's: the issued bf16 MFMAs' cycles at the peak clock over the
        # measured time. The f32-equivalent rate (useful f32 FLOP / s) is a derived figure: the
        # kernel does not run f32 MFMAs, so it is not a fraction of any peak and none is quoted
        return {"roofline": {"bound": "mfma", "unit": "matrix-pipe time", "floor_us": floor_us,
                             "frac": floor_us / us,
                             "what": "864 v_mfma_f32_32x32x16_bf16 (32 cycles) per 64 envs and step on 1,024 "
                                     "SIMDs at 2.4 GHz (bf16 on three-piece splits: f32-level error)"},
                "matrix_pipe_floor_us": floor_us, "matrix_pipe_frac": floor_us / us,
                "derived_f32_equivalent_TFLOPs": flop / (us * 1e-6) / 1e12}
    for name, fused, one in (("one_launch", True, True), ("mfma", True, False), ("torch", False, False)):
        m = PPO(env, PPOConfig(n_steps=args.rollout_steps, fused_policy=fused, fused_rollout=one), seed=0)
        m.collect_rollouts(use_graph=True)  # capture + warm
        rs = m.collect_rollouts(use_graph=True)
        out[name] = {"env_steps_per_s": rs.env_steps / rs.seconds,
                     "ms_per_step": rs.seconds / args.rollout_steps * 1e3}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if one:  # the rollout kernel alone: HIP events on its stream, one launch = n_steps steps
            def launch():
                m._fp.rollout(env, obs_copy=m.buf_obs, actions=m.buf_act, log_prob=m.buf_logp,
                              value=m.buf_val, episode_starts=m.buf_start, rewards=m.buf_rew,
                              last_obs=m.last_obs, last_start=m.last_start, ep_ret=m.ep_ret,
                              ep_len=m.ep_len, stats=m._slots, t0=0, steps=args.rollout_steps,
                              seed=1, gamma=m.cfg.gamma)
            launch()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(3):
                launch()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 3
            flop = flop_step * args.rollout_steps
            out["rollout_kernel"] = {
                "kernel": "k_rollout<HOVER,noCTBR>", "steps_per_launch": args.rollout_steps,
                "kernel_us": us, "us_per_step": us / args.rollout_steps,
                "env_steps_per_s": n * args.rollout_steps / (us * 1e-6),
                "flop_per_launch": flop, **mlp_roofline(flop, us, args.rollout_steps)}
        elif fused:  # the two-launch path's policy kernel alone: MFMA roofline
            ae = torch.empty(n, 4, device=env.device)
            for _ in range(5):
                m._fp.act(m.last_obs, ae, seed=1)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(100):
                m._fp.act(m.last_obs, ae, seed=1)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 100
            out["policy_kernel"] = {"kernel": "k_policy_act<2,256>", "kernel_us": us,
                                    "flop_per_launch": flop_step, **mlp_roofline(flop_step, us, 1)}
        del m
        torch.cuda.empty_cache()
    out["env_steps_per_s"] = out["one_launch"]["env_steps_per_s"]
    # SURVEY config 5 at the PPO level: TrajectoryFollowEnv + RateControlWrapper, the same one-launch
    # rollout (k_rollout<TRAJ, CTBR>) on its own 65,536 envs
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    te = QuadVecEnv(n, env="trajectory", wrapper="RateControlWrapper", device=env.device, seed=args.seed,
                    env_id_base=env.env_id_base)
    m = PPO(te, PPOConfig(n_steps=args.rollout_steps), seed=0)
    m.collect_rollouts(use_graph=True)
    rs = m.collect_rollouts(use_graph=True)
    out["config5_traj_ctbr_one_launch"] = {"env_steps_per_s": rs.env_steps / rs.seconds,
                                           "ms_per_step": rs.seconds / args.rollout_steps * 1e3}
    del m
    te.close()
    torch.cuda.empty_cache()
    return out


def _cpu_info() -> dict:
    """The host the CPU baselines ran on: model name, logical CPUs, and the cores this process may
    use (affinity mask, capped by OMP_NUM_THREADS: the GPU box grants 16 of a larger machine)."""
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        usable = min(usable, int(omp))
    return {"model": model, "logical_cpus": os.cpu_count(), "usable_cores": max(1, usable)}


def _cpu_baseline(seconds: float, threads: int = 1) -> dict:
    """The float64 CPU oracle (C restatement of HoverEnv + MuJoCo's step), SB3 DummyVecEnv order
    (envs stepped one after another), random actions + auto-reset. threads > 1: that many
    independent 64-env batches stepped concurrently (ctypes drops the GIL), SubprocVecEnv-style."""
    import threading
    from oracle import oracle as O
    n_envs = 64
    steps = 200
    t0 = time.perf_counter()
    O.bench_rollout(n_envs, steps, 0)
    dt = time.perf_counter() - t0
    steps = max(200, int(steps * seconds / max(dt, 1e-6)))
    th = [threading.Thread(target=O.bench_rollout, args=(n_envs, steps, k)) for k in range(threads)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    cpu = _cpu_info()
    return {"value": threads * n_envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ float64 C restatement (HoverEnv + MuJoCo-equivalent mj_step + SB3 "
                      f"auto-reset), {threads} x {n_envs} envs x {steps} steps sequential per thread, "
                      f"random actions, {threads} thread(s), {dt:.1f} s on {cpu['model']} "
                      f"({cpu['logical_cpus']} logical CPUs, {cpu['usable_cores']} usable)"}


def _cpu_baseline_ppo(seconds: float, threads: int = 1) -> dict:
    """SURVEY config 1 on the host: the reference's CPU training loop shape -- train.py's 16 envs
    (HoverEnv + RateControlWrapper) stepped one after another (DummyVecEnv) through the float64 C
    oracle, a torch-CPU ActorCritic with SB3 semantics, GAE, and the SB3 update (n_epochs x
    minibatches of 128 rows, clip_grad_norm_, Adam), `threads` torch threads. Bounded: one rollout of
    n_steps and as many update minibatches as fit the time budget, extrapolated per iteration."""
    import numpy as np
    from oracle import oracle as O
    from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic
    from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig, ppo_loss
    old_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        cfg = PPOConfig()
        n_envs, T = 16, cfg.n_steps
        ocfg = O.default_cfg(O.ENV_HOVER, O.WRAP_CTBR)
        envs = [O.Env(cfg=ocfg) for _ in range(n_envs)]
        episode = [0] * n_envs
        obs = np.stack([e.reset_with(*O.reset_draw(ocfg, 0, i, 0)) for i, e in enumerate(envs)])
        torch.manual_seed(0)
        pol = ActorCritic()
        opt = torch.optim.Adam(pol.parameters(), lr=cfg.learning_rate, eps=cfg.adam_eps)
        buf = {k: torch.zeros(T, n_envs, d) for k, d in (("obs", 12), ("act", 4))}
        lp_b, v_b, r_b, s_b = (torch.zeros(T, n_envs) for _ in range(4))
        start = torch.ones(n_envs)
        t0 = time.perf_counter()
        with torch.no_grad():
            for t in range(T):
                o = torch.from_numpy(obs)
                mean, v = pol.forward_heads(o)
                a = mean + pol.log_std.exp() * torch.randn_like(mean)
                buf["obs"][t], buf["act"][t], lp_b[t], v_b[t], s_b[t] = o, a, pol.log_prob(mean, a), v, start
                ac = a.clamp(-1, 1).numpy()
                for i, e in enumerate(envs):
                    out = e.step(ac[i])
                    r = float(out.reward)
                    if out.truncated and not out.terminated:  # TimeLimit bootstrap
                        r += cfg.gamma * float(pol.value(torch.from_numpy(np.array(out.obs[:], np.float32))[None])[0])
                    r_b[t, i] = r
                    done = bool(out.terminated or out.truncated)
                    start[i] = float(done)
                    if done:
                        episode[i] += 1
                        obs[i] = e.reset_with(*O.reset_draw(ocfg, 0, i, episode[i]))
                    else:
                        obs[i] = np.array(out.obs[:], np.float32)
            last_v = pol.value(torch.from_numpy(obs))
        adv, ret = torch.zeros(T, n_envs), torch.zeros(T, n_envs)
        gae_acc = torch.zeros(n_envs)
        for t in reversed(range(T)):  # SB3 RolloutBuffer.compute_returns_and_advantage
            nv, nnt = (last_v, 1.0 - start) if t == T - 1 else (v_b[t + 1], 1.0 - s_b[t + 1])
            delta = r_b[t] + cfg.gamma * nv * nnt - v_b[t]
            gae_acc = delta + cfg.gamma * cfg.gae_lambda * nnt * gae_acc
            adv[t] = gae_acc
        ret = adv + v_b
        t_roll = time.perf_counter() - t0
        M, B = T * n_envs, 128
        flat = [buf["obs"].view(M, 12), buf["act"].view(M, 4), lp_b.view(M), adv.view(M), ret.view(M)]
        steps_total = cfg.n_epochs * (M // B)
        t1, done = time.perf_counter(), 0
        budget = max(1.0, seconds - t_roll)
        while done < steps_total and time.perf_counter() - t1 < budget:
            idx = torch.randperm(M)[:B]
            loss = ppo_loss(pol, *[x[idx] for x in flat], cfg)[0]
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(pol.parameters(), cfg.max_grad_norm)
            opt.step()
            done += 1
        t_upd = (time.perf_counter() - t1) * steps_total / max(done, 1)
        it = t_roll + t_upd
        return {"value": M / it, "unit": "env-steps/s (whole PPO iteration)", "cores": threads, "kind": "port",
                "sample": f"train.py loop on the host: 16 oracle envs (HoverEnv + RateControlWrapper, DummyVecEnv "
                          f"order) x {T} steps + torch-CPU PPO update (SB3 schedule: {steps_total} Adam steps of "
                          f"{B} rows; {done} timed, extrapolated), {threads} torch thread(s); rollout {t_roll:.1f} s, update "
                          f"{t_upd:.1f} s per iteration"}
    finally:
        torch.set_num_threads(old_threads)


def _pmc_traffic(symbol: str, n_envs: int):
    """HBM-side bytes per launch of THIS kernel at this size from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc/traffic_summary.py, keyed by kernel symbol and env count),
    or None when no pass of the kernel the bench timed exists."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        rec = d.get("kernels", {}).get(symbol, {}).get(str(n_envs))
        if not rec:
            return None
        return {"bytes_per_launch": rec["hbm_bytes_per_launch"], "kernel": symbol, "envs": n_envs,
                "traffic_over_algorithmic": rec["traffic_over_algorithmic"], "round": d.get("round"),
                "source": "profiles/pmc_traffic.json"}
    except Exception:
        return None


def _pmc_issue(symbol: str, n_envs: int):
    """The timed kernel's counted issue roofline (rocprofv3 PMC: instruction counts by class,
    SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / wait shares, GRBM_GUI_ACTIVE per launch) from the committed
    summary (tools/pmc/issue_roofline.py -> profiles/pmc_issue.json, keyed by kernel symbol and env
    count, like the traffic file), or None when no pass of the kernel the bench timed exists."""
    path = os.path.join(REPO, "profiles", "pmc_issue.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        rec = d.get("kernels", {}).get(symbol, {}).get(str(n_envs))
        if not rec:
            return None
        return dict(rec, kernel=symbol, envs=n_envs, round=d.get("round"), source="profiles/pmc_issue.json")
    except Exception:
        return None


def _launch_ranks(args) -> int:
    """`--gpus N` without a torch.distributed launcher: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, one GPU each) and return their exit status. This parent never makes
    a HIP call; if a rank fails, the others are stopped instead of waiting at a barrier."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def _check_launch(args, rank: int, world: int) -> None:
    """--check-launch: the rank topology alone, on gloo (no GPU): every rank joins, the world
    size matches --gpus, an all_reduce of the ranks reaches everyone; rank 0 prints one line."""
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        ranks_sum = float(t.item())
        dist.barrier()
        dist.destroy_process_group()
    else:
        ranks_sum = 0.0
    if rank == 0:
        print(json.dumps({"check_launch": True, "n_gpus": world, "ranks_sum": ranks_sum,
                          "global_envs": args.envs * world}), flush=True)


def _launch_terms(res, envs: int) -> dict:
    """The one-launch step against its dispatch floor: the HBM fraction of the time beyond the
    empty-kernel launch cost, and the ceiling a one-launch step of these bytes could reach (a
    zero-latency kernel moving them at the peak: bytes / peak / (bytes / peak + floor))."""
    fl = res.get("launch_floor_us")
    if not fl:
        return {}
    byt = BYTES_PER_ENV_STEP * envs
    at_peak_us = byt / (HBM_PEAK_GBS * 1e3)
    beyond = res["kernel_us"] - fl
    return {"launch_floor_us": fl,
            "frac_beyond_launch_floor": (byt / (beyond * 1e-6) / 1e9) / HBM_PEAK_GBS if beyond > 0 else None,
            "frac_ceiling_one_launch": at_peak_us / (at_peak_us + fl)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=ENVS_PER_GPU)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graph-chunk", type=int, default=100)
    ap.add_argument("--action-batches", type=int, default=256)
    ap.add_argument("--kernel-launches", type=int, default=200)
    ap.add_argument("--large-envs", type=int, default=1 << 20)
    ap.add_argument("--dram-envs", type=int, default=1 << 22)
    ap.add_argument("--cpu-seconds", type=float, default=7.0)
    ap.add_argument("--rollout-steps", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true")
    ap.add_argument("--e2e-iters", type=int, default=1)
    ap.add_argument("--e2e-steps", type=int, default=1024)
    ap.add_argument("--e2e-epochs", type=int, default=20)
    ap.add_argument("--check-launch", action="store_true",
                    help="test the rank launch only (gloo, no GPU)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args))  # one child per GPU; this process never touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    if args.check_launch:
        return _check_launch(args, rank, world)
    # rehearsal knob (tests only): run all ranks on one GPU over gloo, e.g. 2 ranks on a 1-GPU box
    rehearsal = os.environ.get("QUAD_BENCH_REHEARSAL") == "1"
    device_index = 0 if rehearsal else local_rank
    if not rehearsal and torch.cuda.device_count() < local_rank + 1:
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local_rank}, "
                         f"{torch.cuda.device_count()} visible")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(device_index)
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
        assert dist.get_world_size() == args.gpus

    res = _run_rank(args, rank, world, device_index)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return
    n_total = args.envs * world
    value = n_total * args.steps / res["elapsed"]
    kus = res["kernel_us"]
    achieved = BYTES_PER_ENV_STEP * args.envs / (kus * 1e-6) / 1e9
    traffic = _pmc_traffic(res["symbol"], args.envs)
    line = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": res["elapsed"] / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": "HoverEnv step + SB3 auto-reset, random actions pre-generated in "
                               "HBM (configs[1] step-kernel-only shape at the metric's 65,536 "
                               "envs/GPU), hipGraph replay",
                   "envs_per_gpu": args.envs, "global_envs": n_total,
                   "parallelism": f"env-shard x{world} (no data-path collective)"},
        "device_us_per_step": res["region_us"],
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic["bytes_per_launch"] if traffic else None, "traffic_pmc": traffic,
                     "kernel": res["kernel"], "kernel_symbol": res["symbol"], "kernel_us": kus,
                     "algorithmic_bytes_per_launch": BYTES_PER_ENV_STEP * args.envs,
                     "issue": _pmc_issue(res["symbol"], args.envs), **_launch_terms(res, args.envs)},
    }
    if "per_rank" in res:
        line["per_rank"] = res["per_rank"]
    if "rollout" in res:
        line["rollout_phase"] = res["rollout"]
    if "end_to_end" in res:
        line["end_to_end"] = res["end_to_end"]
    if "configs" in res:
        line["configs"] = res["configs"]
    if "large" in res:
        line["large_batch"] = dict(res["large"], note="working set ~290 MB: Infinity-Cache assisted, not a DRAM figure")
    if "dram" in res:
        line["large_batch_dram"] = dict(res["dram"], note="1.2 GB per launch (4.5x the 256 MB Infinity Cache): "
                                                          "the step's true HBM roofline point")
    if not args.no_cpu_baseline and world == 1:
        cores = _cpu_info()["usable_cores"]
        line["cpu_host"] = _cpu_info()
        line["cpu_baseline"] = _cpu_baseline(args.cpu_seconds, 1)
        line["cpu_baseline_all_cores"] = _cpu_baseline(args.cpu_seconds, cores)
        line["cpu_baseline_ppo"] = _cpu_baseline_ppo(args.cpu_seconds, 1)
        line["cpu_baseline_ppo_all_cores"] = _cpu_baseline_ppo(args.cpu_seconds, cores)
    line["summary"] = _summary(line)  # last: the driver keeps the tail of stdout
    print(json.dumps(line), flush=True)


def _summary(line: dict) -> dict:
    """The line's key figures in a few hundred bytes, printed as its last key (the driver records
    only the last 2,000 characters of stdout; the full objects above precede it)."""
    def g(*path):
        x = line
        for k in path:
            if not isinstance(x, dict) or k not in x:
                return None
            x = x[k]
        return round(x, 4) if isinstance(x, float) else x
    return {
        "step_value": g("value"), "step_kernel_us": g("roofline", "kernel_us"), "step_frac": g("roofline", "frac"),
        "step_frac_beyond_launch_floor": g("roofline", "frac_beyond_launch_floor"),
        "launch_floor_us": g("roofline", "launch_floor_us"),
        "rollout_env_steps_per_s": g("rollout_phase", "env_steps_per_s"),
        "rollout_kernel_us_per_step": g("rollout_phase", "rollout_kernel", "us_per_step"),
        "rollout_matrix_pipe_frac": g("rollout_phase", "rollout_kernel", "matrix_pipe_frac"),
        "e2e_env_steps_per_s": g("end_to_end", "env_steps_per_s"), "e2e_train_s": g("end_to_end", "train_s"),
        "e2e_rollout_s": g("end_to_end", "rollout_s"),
        "learner_us_per_minibatch": g("end_to_end", "learner_kernel", "us_per_minibatch"),
        "learner_matrix_pipe_frac": g("end_to_end", "learner_kernel", "matrix_pipe_frac"),
        "large_1M_kernel_us": g("large_batch", "kernel_us"), "large_1M_frac": g("large_batch", "frac"),
        "dram_4M_kernel_us": g("large_batch_dram", "kernel_us"), "dram_4M_frac": g("large_batch_dram", "frac"),
        "dram_4M_copy_floor_us": g("large_batch_dram", "copy_floor_us"),
        "dram_4M_frac_of_copy_floor": g("large_batch_dram", "frac_of_copy_floor"),
        "config2_4096_one_launch_us_per_step": g("configs", "config2_hover_4096_one_launch", "us_per_step"),
        "config5_traj_ctbr_us": g("configs", "config5_traj_ctbr_65536", "kernel_us"),
        "config1_on_gpu_env_steps_per_s": g("configs", "config1_train_py_on_gpu", "env_steps_per_s"),
        "cpu_baseline": g("cpu_baseline", "value"), "cpu_baseline_ppo": g("cpu_baseline_ppo", "value"),
        "per_rank_elapsed_max_over_min": g("per_rank", "elapsed_s", "max_over_min"),
        "per_rank_slowest": g("per_rank", "elapsed_s", "argmax_rank"),
        "allreduce_median_us": g("end_to_end", "allreduce", "median_us"),
    }


if __name__ == "__main__":
    main()
