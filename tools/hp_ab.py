#!/usr/bin/env python3
"""Profiling tool (not product; with tools/patches/step_hp_persistent_prefetch.patch applied, round 6 A/B,
not kept: profiles/r06/step_hp_ab.txt): the DRAM-size step forms A/B -- k_step_hd (QUADENV_HD=1) vs the
persistent prefetching k_step_hp (QUADENV_HD=2) -- per library build (tools/hp_build.sh), beside
quad_mem_floor on the same buffers. Graph-replayed launches, HIP events, alternating, best of 3.
Usage: hp_ab.py lib1.so [lib2.so ...]   (env HP_SIZES="4194304,8388608")"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, n):
    sys.path.insert(0, ROOT)
    import torch
    from uav_reinforcement_learning_control_amd import _native as N
    N.LIB_PATH = lib
    from uav_reinforcement_learning_control_amd.envs import QuadVecEnv
    from bench import _quad_step_fn, _mem_floor_fn, _gated_kernel_us
    res = {}
    for rep in range(3):
        for hd in ("1", "2"):
            os.environ["QUADENV_HD"] = hd
            e = QuadVecEnv(n, env="hover", device="cuda:0", seed=0)
            e.reset()
            acts = [e.random_actions(k) for k in range(8)]
            st = _quad_step_fn(e)
            for k in range(30):
                st(acts[k % 8].data_ptr())
            us = _gated_kernel_us(st, acts, 40)
            form = int(N.lib().quad_kernel_form(e._h))
            if hd == "1":
                res.setdefault("floor", []).append(_gated_kernel_us(_mem_floor_fn(e), acts, 40))
            res.setdefault(f"hd{hd}", []).append(us)
            res.setdefault(f"form{hd}", form)
            e.close()
            del acts
            torch.cuda.empty_cache()
    import hashlib
    dig = {}
    for hd in ("1", "2"):  # same bits: 6 steps from the same reset, every output and the final state
        os.environ["QUADENV_HD"] = hd
        e = QuadVecEnv(n, env="hover", device="cuda:0", seed=3)
        h = hashlib.sha256()
        h.update(e.reset().cpu().numpy().tobytes())
        for k in range(6):
            obs, rew, te, tr, inf = e.step(e.random_actions(k))
            for x in (obs, rew, te, tr, inf["terminal_observation"]):
                h.update(x.cpu().numpy().tobytes())
        for k2, v in sorted(e.get_state().items()):
            h.update(v.tobytes())
        dig[hd] = h.hexdigest()[:16]
        e.close()
        torch.cuda.empty_cache()
    res["digest_hd"], res["digest_hp"] = dig["1"], dig["2"]
    print(json.dumps({"lib": os.path.basename(lib), "envs": n, **{k: (min(v) if isinstance(v, list) else v) for k, v in res.items()},
                      "all": res}), flush=True)


def main():
    if sys.argv[1] == "child":
        return child(sys.argv[2], int(sys.argv[3]))
    sizes = [int(x) for x in os.environ.get("HP_SIZES", "4194304").split(",")]
    for n in sizes:
        for lib in sys.argv[1:]:
            r = subprocess.run([sys.executable, __file__, "child", lib, str(n)], capture_output=True, text=True, timeout=400)
            print(r.stdout.strip() or r.stderr.strip()[-800:], flush=True)
            if r.returncode:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
