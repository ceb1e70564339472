"""Diagnostic (not product): per-tensor error of both quad_ppo_grad forms vs float64 autograd,
on all rows and on the rows whose hidden pre-activations are all >= eps away from zero."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_learner import _policy, _buffers, _torch_grads  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.learner import FusedLearner, _ordered  # noqa: E402
from uav_reinforcement_learning_control_amd.ppo.ppo import PPOConfig  # noqa: E402

names = ["pi_w0", "pi_b0", "pi_w1", "pi_b1", "act_w", "act_b", "vf_w0", "vf_b0", "vf_w1", "vf_b1", "val_w", "val_b", "log_std"]
cfg = PPOConfig()


def margin(pol, x):
    x = x.double()
    ex = pol.mlp_extractor
    m = torch.full((x.shape[0],), float("inf"), dtype=torch.float64, device=x.device)
    for net in (ex.policy_net, ex.value_net):
        h1 = x @ net[0].weight.double().T + net[0].bias.double()
        h2 = torch.relu(h1) @ net[2].weight.double().T + net[2].bias.double()
        m = torch.minimum(m, torch.minimum(h1.abs().min(1).values, h2.abs().min(1).values))
    return m


for M, B in [(80000, 65536), (300000, 262144)]:
    pol = _policy(5)
    obs, act, logp_old, adv, ret = _buffers(pol, M, 5, cfg.clip_range)
    idx0 = torch.randperm(M, generator=torch.Generator().manual_seed(14))[:B].cuda()
    mg = margin(pol, obs[idx0])
    for eps in (0.0, 1e-5):
        idx = idx0[mg >= eps].contiguous()
        ref64, _ = _torch_grads(pol, torch.float64, obs, act, logp_old, adv, ret, idx, cfg)
        ref32, _ = _torch_grads(pol, torch.float32, obs, act, logp_old, adv, ret, idx, cfg)
        res = {}
        for form in ("x3", "f32"):
            if form == "f32":
                os.environ["QUADENV_LEARNER"] = "f32"
            else:
                os.environ.pop("QUADENV_LEARNER", None)
            fl = FusedLearner(pol, cfg.clip_range, cfg.ent_coef, cfg.vf_coef, True)
            fl.grads(obs, act, logp_old, adv, ret, idx, None)
            torch.cuda.synchronize()
            res[form] = [p.grad.double().clone() for p in _ordered(pol)]
        print(f"B={B} eps={eps}: {idx.numel()} rows (min margin {mg.min().item():.2e})")
        for i, n in enumerate(names):
            sc = ref64[i].abs().max().item()
            e = {f: (res[f][i] - ref64[i]).abs().max().item() / sc for f in res}
            e32 = (ref32[i] - ref64[i]).abs().max().item() / sc
            print(f"  {n:8s} x3 {e['x3']:.2e}  f32 {e['f32']:.2e}  torch32 {e32:.2e}")
