#!/usr/bin/env python3
"""Step-kernel cost ablation at N envs: auto-reset on/off (random actions reset ~10 % of envs per
step, so nearly every wave runs the reset branch), and calm actions (no resets) -- graph-replayed,
HIP-event timed. Prints JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import _quad_step_fn  # noqa: E402
from uav_reinforcement_learning_control_amd.envs import QuadVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536


def timed(env, acts, reps=20, per=20):
    st = _quad_step_fn(env)
    for k in range(30):
        st(acts[k % len(acts)].data_ptr())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(per):
            st(acts[k % len(acts)].data_ptr())
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * per)


res = {"n": n}
for name, auto, calm in (("random_autoreset", True, False), ("random_noreset", False, False),
                         ("calm_autoreset", True, True)):
    env = QuadVecEnv(n, env="hover", device="cuda:0", seed=1, auto_reset=auto)
    env.reset()
    if calm:  # hover thrust, zero torque: nothing terminates within the timed steps
        a = torch.tensor([[-0.915, 0.0, 0.0, 0.0]], device="cuda").repeat(n, 1)
        acts = [a]
    else:
        acts = [env.random_actions(k) for k in range(16)]
    res[name] = timed(env, acts)
    env.close()
print(json.dumps(res))
