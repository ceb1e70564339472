#!/usr/bin/env python3
"""Profiling tool (not product): a rocprofv3 kernel-trace CSV summarized per (kernel, grid size) --
rocprofv3's --stats groups by kernel name only, and since round 4 one step-kernel symbol
(k_step_h<0, false, true, 256, true>) runs both the 65,536-env headline grid and the 4M-env DRAM
grid of the same bench command. Usage: trace_by_grid.py run_kernel_trace.csv [regex] > out.csv"""
import csv
import re
import statistics
import sys


def main(path, pat=r"k_step|k_ppo_grad|k_rollout|k_policy"):
    rx = re.compile(pat)
    groups = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not rx.search(name):
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        groups.setdefault((name, grid), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "GridThreads", "Calls", "MeanUs", "MedianUs", "MinUs", "MaxUs"])
    for (name, grid), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, grid, len(d), round(statistics.mean(d), 3), round(statistics.median(d), 3),
                    round(min(d), 3), round(max(d), 3)])


if __name__ == "__main__":
    main(*sys.argv[1:])
