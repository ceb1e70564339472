#!/usr/bin/env python3
"""Time the MFMA policy kernel alone (HIP events, graph-free) at N envs: pure policy evaluation,
and with the fused epilogue (pending step, no timeouts / all timeouts). Prints JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from uav_reinforcement_learning_control_amd import _native as N  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
pol = ActorCritic().cuda()
fp = FusedPolicy(pol)
fp.pack()
T = 16
f = lambda *s: torch.zeros(*s, device="cuda")
obs = torch.rand(n, 12, device="cuda") * 2 - 1
ae, act, lp, val, oc, st = f(n, 4), f(T, n, 4), f(T, n), f(T, n), f(T, n, 12), f(T, n)
rew, ls, er, el, tobs = f(n), f(n), f(n), f(n), f(n, 12)
tfalse = torch.zeros(n, dtype=torch.bool, device="cuda")
ttrue = torch.ones(n, dtype=torch.bool, device="cuda")
slots = torch.zeros(N.POLICY_STAT_SLOTS, 3, dtype=torch.float64, device="cuda")
cur = torch.zeros(4, dtype=torch.int32, device="cuda")
epi_none = fp.make_epilogue(rew, tfalse, tfalse, tobs, f(T, n), ls, er, el, slots, T, 0.99)
epi_all = fp.make_epilogue(rew, tfalse, ttrue, tobs, f(T, n), ls, er, el, slots, T, 0.99)
kw = dict(actions=act, log_prob=lp, value=val, obs_copy=oc, last_start=ls, episode_starts=st,
          cursor=cur, rows=T, seed=1)


def timed(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


res = {"n": n}
res["act_us"] = timed(lambda: fp.act(obs, ae, **kw))
res["act_epilogue_us"] = timed(lambda: fp.act(obs, ae, epilogue=epi_none, **kw))
res["act_epilogue_all_timeouts_us"] = timed(lambda: fp.act(obs, ae, epilogue=epi_all, **kw))
flop = n * 2 * 2 * (12 * 128 + 128 * 128) + n * 2 * (128 * 5)
res["tflops_act"] = flop / (res["act_us"] * 1e-6) / 1e12
print(json.dumps(res))
