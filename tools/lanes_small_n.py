#!/usr/bin/env python3
"""Profiling tool (not product): step-kernel forms (QUADENV_LANES 0/1/2/4) at small batches (4,096 /
16,384 / 65,536 envs), one process per point, graph-replayed, HIP-event timed (tools/lanes_sweep.run)."""
import os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
if len(sys.argv) > 1:
    from lanes_sweep import run
    lanes, n = int(sys.argv[1]), int(sys.argv[2])
    print(f"lanes={lanes} n={n}: {run(lanes, n, steps=400):.2f} us", flush=True)
else:
    for n in (4096, 16384, 65536):
        for lanes in (0, 1, 2, 4):
            r = subprocess.run([sys.executable, __file__, str(lanes), str(n)], capture_output=True, text=True)
            print(r.stdout.strip() or r.stderr[-300:], flush=True)
