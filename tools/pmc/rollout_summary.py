#!/usr/bin/env python3
"""Summarize tools/pmc/rollout_pmc.sh (gpurun_out/ro_pmc/p*/) into a JSON profile of k_rollout:
per-dispatch counters, the effective clock, the matrix-pipe busy fraction and the wave-cycle split
(units as tools/pmc/learner_summary.py). Usage: rollout_summary.py OUT.json"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(out):
    per, dur, name = defaultdict(list), [], None
    for f in sorted(glob.glob("gpurun_out/ro_pmc/p*/**/*counter_collection.csv", recursive=True)):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
        for r in rows:
            if "k_rollout" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    drop = lambda v: v[1:] if len(v) > 1 else v  # the warm launch
    avg = {c: sum(drop(v)) / len(drop(v)) for c, v in per.items()}
    us = sorted(drop(dur))[len(drop(dur)) // 2]
    clock = avg["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3)
    waves = avg["SQ_WAVES"]
    res = {"kernel": name, "launch": "65,536 hover envs x 64 steps", "kernel_us_profiled_median": us,
           "us_per_step": us / 64, "clock_GHz": clock, "counters_per_dispatch": avg,
           "per_wave": {c: avg[c] / waves for c in avg if c.startswith("SQ_") and c != "SQ_WAVES"},
           "mfma_per_wave_per_step": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / waves / 32 / 64,
           "matrix_pipe_busy_frac": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (us * 1e3 * clock),
           "wave_cycle_split": {k: avg[c] / avg["SQ_WAVE_CYCLES"] for k, c in
                                (("waiting", "SQ_WAIT_ANY"), ("issue_stalled", "SQ_WAIT_INST_ANY"),
                                 ("issuing", "SQ_ACTIVE_INST_ANY"), ("valu", "SQ_ACTIVE_INST_VALU"))}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("counters_per_dispatch", "per_wave")}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
