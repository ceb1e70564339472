#!/usr/bin/env python3
"""Profiling tool (not product): graph-replayed step-kernel time (HIP events, tools/lanes_sweep.run)
at several batch sizes and step forms, with the algorithmic GB/s (278 B per env-step)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lanes_sweep import run  # noqa: E402

out = []
for n, forms in ((65536, (0, 1)), (1048576, (0, 1, 2)), (4194304, (1, 2))):
    for lanes in forms:
        us = run(lanes, n, steps=200 if n < 4194304 else 100)
        out.append({"envs": n, "lanes": lanes, "us": us, "GBs": 278.0 * n / us / 1e3})
        print(json.dumps(out[-1]), flush=True)
