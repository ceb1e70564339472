#!/usr/bin/env python3
"""Profiling tool (not product): A/B whole-library builds on the step kernel -- `k_step_h`
graph-replayed at N envs with each .so given on the command line (one process per library, the
in-tree library as "base"). Usage: lib_ab.py N lib1.so [lib2.so ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    if sys.argv[1] == "child":
        sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
        from uav_reinforcement_learning_control_amd import _native as N
        if sys.argv[3] != "base":
            N.LIB_PATH = sys.argv[3]
        from step_time import run
        print(f"{os.path.basename(sys.argv[3]):16s} n={sys.argv[2]}: {run(int(sys.argv[2]), steps=1000):.2f} us", flush=True)
        return
    n = sys.argv[1]
    for lib in ["base"] + sys.argv[2:] + ["base"]:
        r = subprocess.run([sys.executable, __file__, "child", n, lib], capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-300:], flush=True)


if __name__ == "__main__":
    main()
