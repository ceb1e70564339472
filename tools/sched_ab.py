#!/usr/bin/env python3
"""Profiling tool (not product): step-kernel time of library variants (tools/sched_ab.sh), one
process per library (QUADENV_LIB), interleaved twice: k_step_h at 65,536 envs, k_step_g<1> at 1M and 4M."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
    from step_time import run
    print(f"{os.path.basename(os.environ['QUADENV_LIB']):18s} 65536: {run(65536, steps=1000):.3f} us   "
          f"1M: {run(1048576, steps=200):.2f} us   4M: {run(4194304, steps=100):.1f} us", flush=True)
    sys.exit(0)
libs = sys.argv[1:]
for rep in range(2):
    for lib in libs:
        env = dict(os.environ, QUADENV_LIB=os.path.join(ROOT, lib))
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=300)
        print(r.stdout.strip() or r.stderr.strip()[-300:], flush=True)
