#!/usr/bin/env python3
"""Comparison (tools only, not product): the plain LDS-tiled f32 VALU policy forward
(tools/valu_policy/valu_policy.hip, built to tools/_build/libvalu_policy.so) against the MFMA policy
kernel k_policy_act (csrc/policy.hip) at N envs -- the north star's "MFMA only if it beats a plain
LDS-tiled kernel" check. Both are checked against torch fp32 on the same inputs; HIP-event timed.
k_policy_act additionally samples the Gaussian, forms log-probs and writes the buffer rows.
Usage: valu_policy_bench.py [N] [reps]. Prints JSON."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from uav_reinforcement_learning_control_amd import _native as N  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.fused import FusedPolicy  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.learner import _ordered  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.policy import ActorCritic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
torch.manual_seed(0)
pol = ActorCritic().cuda()
with torch.no_grad():
    for name, p in pol.named_parameters():
        if name.endswith("bias"):
            p.copy_(torch.randn_like(p) * 0.1)
obs = torch.rand(n, 12, device="cuda") * 2 - 1
lib = C.CDLL(os.path.join(ROOT, "tools", "_build", "libvalu_policy.so"))
VARIANTS = ("u4", "u8", "u16", "p4", "p8")  # k-loop unroll 4/8/16; p = operands of k+1 loaded before k's FMAs
for v in VARIANTS:
    getattr(lib, "valu_policy_" + v).argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                                  C.c_void_p]
ps = _ordered(pol)[:12]  # pi: w0 b0 w1 b1 act_w act_b; vf: w0 b0 w1 b1 val_w val_b
ptrs = (C.c_void_p * 12)(*[p.data_ptr() for p in ps])
mean = torch.empty(n, 4, device="cuda")
value = torch.empty(n, device="cuda")
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def timed(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


with torch.no_grad():
    ref_mean, ref_v = pol.forward_heads(obs)
flop = n * 2 * 2 * (12 * 128 + 128 * 128) + n * 2 * (128 * 5)
res = {"n": n, "flop": flop, "valu": {}}
for v in VARIANTS:
    fn = getattr(lib, "valu_policy_" + v)
    for nb in (128, 256):
        call = lambda: fn(ptrs, C.c_void_p(obs.data_ptr()), n, C.c_void_p(mean.data_ptr()),
                          C.c_void_p(value.data_ptr()), nb, stream)
        mean.zero_(); value.zero_()
        assert call() == 0
        torch.cuda.synchronize()
        err = max(((mean - ref_mean).abs() / (1 + ref_mean.abs())).max().item(),
                  ((value - ref_v.reshape(-1)).abs() / (1 + ref_v.reshape(-1).abs())).max().item())
        us = timed(call)
        res["valu"][f"{v}/{nb}"] = {"us": us, "TFLOPs": flop / us / 1e6, "max_rel_err_vs_torch": err}
best = min(res["valu"].items(), key=lambda kv: kv[1]["us"])
res["valu_best"] = {"variant": best[0], **best[1]}

# the MFMA kernel (k_policy_act: forward + Gaussian sample + log-prob + buffer rows)
fp = FusedPolicy(pol)
fp.pack()
T = 16
f = lambda *s: torch.zeros(*s, device="cuda")
ae, act, lp, val, oc, st, ls = f(n, 4), f(T, n, 4), f(T, n), f(T, n), f(T, n, 12), f(T, n), f(n)
cur = torch.zeros(4, dtype=torch.int32, device="cuda")
kw = dict(actions=act, log_prob=lp, value=val, obs_copy=oc, last_start=ls, episode_starts=st, cursor=cur, rows=T,
          seed=1)
fp.act(obs, ae, **kw)
torch.cuda.synchronize()
verr = ((val[0] - ref_v.reshape(-1)).abs() / (1 + ref_v.reshape(-1).abs())).max().item()
us = timed(lambda: fp.act(obs, ae, **kw))
res["mfma_k_policy_act"] = {"us": us, "TFLOPs": flop / us / 1e6, "max_rel_err_value_vs_torch": verr}
print(json.dumps(res))
