#!/usr/bin/env python3
"""Profiling tool (not product): A/B of whole-library builds on the one-thread step form (k_step_h
below 262,144 envs) -- per library (QUADENV_LIB, one process each, interleaved twice) the
graph-replayed step time at 4,096 and 65,536 envs (tools/step_time.run) and a digest of every
output of 300 stepped steps (obs, reward, flags, terminal obs, state) for each env kind, so that
a faster variant is also shown to give the same bits. Usage: lib_digest_ab.py lib1.so [lib2.so ...]
("base" = the in-tree library)."""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def digest(env_name, wrapper, info, n=65536, steps=300):
    import torch
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    e = QuadVecEnv(n, env=env_name, wrapper=wrapper, device="cuda:0", seed=3)
    e.reset()
    h = hashlib.sha256()
    for k in range(steps):
        obs, rew, term, trunc, inf = e.step(e.random_actions(k), info=info)
        for t in (obs, rew, term, trunc, inf["terminal_observation"]):
            h.update(t.cpu().numpy().tobytes())
        if info == "full":
            for key in ("motor_commands", "voltage_scale", "state", "target"):
                h.update(inf[key].cpu().numpy().tobytes())
    for v in e.get_state().values():
        h.update(v.tobytes())
    torch.cuda.synchronize()
    e.close()
    return h.hexdigest()[:16]


def child():
    sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
    from step_time import run
    t = [min(run(n, steps=1000) for _ in range(3)) for n in (4096, 65536)]
    d = [digest("hover", None, "basic"), digest("hover", "RateControlWrapper", "full"),
         digest("trajectory", None, "full"), digest("trajectory", "RateControlWrapper", "basic")]
    import torch
    import bench
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    dev = torch.device("cuda", 0)
    kr = [bench._kstep_rate(n, k, dev, 0)["us_per_step"] for n, k in ((4096, 1000), (65536, 200))]
    e = QuadVecEnv(4096, env="hover", device=dev, seed=5)
    e.reset()
    r = e.step_random(300, actions=True)
    h = hashlib.sha256()
    for k in sorted(r):
        h.update(r[k].cpu().numpy().tobytes())
    for v in e.get_state().values():
        h.update(v.tobytes())
    e.close()
    print(f"{os.path.basename(os.environ.get('QUADENV_LIB', 'base')):18s} 4096: {t[0]:.3f} us  "
          f"65536: {t[1]:.3f} us  K-step 4096: {kr[0]:.3f}  65536: {kr[1]:.3f} us/step  "
          f"digests {' '.join(d)} {h.hexdigest()[:16]}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        return child()
    for rep in range(2):
        for lib in sys.argv[1:]:
            env = dict(os.environ)
            if lib != "base":
                env["QUADENV_LIB"] = os.path.join(ROOT, lib)
            r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True,
                               timeout=300)
            print(r.stdout.strip() or r.stderr.strip()[-400:], flush=True)


if __name__ == "__main__":
    main()
