#!/usr/bin/env python3
"""Profiling tool (not product): the step kernel with random actions (about 16 % of waves hold a
resetting env each step) against near-hover actions (no terminations, so no reset branch runs):
the straggler cost of the auto-reset branch. Usage: reset_cost.py N [lanes]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from step_time import run  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
r = sorted(run(n, steps=1000) for _ in range(3))[0]
h = sorted(run(n, steps=1000, hover_actions=True) for _ in range(3))[0]
print(f"n={n} lanes={lanes}: random actions {r:.2f} us/step, near-hover actions (no resets) {h:.2f} us/step")
