#!/usr/bin/env python3
"""Profiling tool (not product): A/B whole-library builds on one step-kernel form at several batch
sizes -- graph-replayed launches, HIP events (tools/lanes_sweep.run), one process per library, the
in-tree library as "base" first and last. Usage: ab_lanes.py LANES N1,N2 lib1.so [lib2.so ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "child":
        sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
        from uav_reinforcement_learning_control_amd import _native as N
        if sys.argv[4] != "base":
            N.LIB_PATH = sys.argv[4]
        from lanes_sweep import run
        lanes = int(sys.argv[2])
        for n in sys.argv[3].split(","):
            n = int(n)
            us = run(lanes, n, steps=200 if n < 4000000 else 100)
            print(f"{os.path.basename(sys.argv[4]):20s} lanes={lanes} n={n}: {us:.2f} us = {278 * n / us / 1e3:.0f} GB/s",
                  flush=True)
        return
    for lib in ["base"] + sys.argv[3:] + ["base"]:
        r = subprocess.run([sys.executable, __file__, "child", sys.argv[1], sys.argv[2], lib],
                           capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-300:], flush=True)


if __name__ == "__main__":
    main()
