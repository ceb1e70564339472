#!/usr/bin/env python3
"""Profiling tool (not product): graph-replayed step-kernel time (HIP events, tools/step_time.run)
at several batch sizes (each size's default kernel form), with the algorithmic GB/s (278 B per
env-step)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_time import run  # noqa: E402

out = []
for n in (4096, 65536, 1048576, 2097152, 4194304):
    us = run(n, steps=200 if n < 4194304 else 100)
    out.append({"envs": n, "us": us, "GBs": 278.0 * n / us / 1e3})
    print(json.dumps(out[-1]), flush=True)
