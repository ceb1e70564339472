#!/usr/bin/env python3
"""Profiling tool (not product): the per-update overheads around quad_ppo_grad at config 3 --
torch.randperm over the 67M-row buffer (once per epoch) and the per-optimizer-step small launches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

n = 65536 * 1024
for _ in range(2):
    torch.randperm(n, device="cuda")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    torch.randperm(n, device="cuda")
e1.record()
torch.cuda.synchronize()
print(f"torch.randperm({n}) on the GPU: {e0.elapsed_time(e1) / 5:.2f} ms")
