#!/usr/bin/env python3
"""Summarize tools/pmc/learner_pmc.sh output (gpurun_out/lrn_pmc_<form>/p*/) into a JSON profile:
per-dispatch counters of the learner kernel (k_ppo_grad_x3 or k_ppo_grad), the wave-cycle split and
the matrix-pipe busy fraction. Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles per wave; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over the
SIMDs; GRBM_GUI_ACTIVE counts GPU cycles of the dispatch (per XCD, summed over the 8 XCDs).
Usage: learner_summary.py OUT.json [form ...]"""
import csv
import glob
import json
import sys
from collections import defaultdict


def summarize(form):
    per = defaultdict(list)
    dur = []
    name = None
    for f in sorted(glob.glob(f"gpurun_out/lrn_pmc_{form}/p*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "ppo_grad" not in k:
                continue
            name = k
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    if not per:
        return None
    avg = {c: sum(v) / len(v) for c, v in per.items()}
    waves = avg["SQ_WAVES"]
    us = sorted(dur)[len(dur) // 2]
    clock_ghz = avg["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3)
    simds = 1024
    out = {"kernel": name, "dispatches": len(per["SQ_WAVES"]), "kernel_us_profiled_median": us,
           "clock_GHz": clock_ghz, "counters_per_dispatch": avg,
           "per_wave": {c: avg[c] / waves for c in avg if c.startswith("SQ_") and c != "SQ_WAVES"},
           "matrix_pipe_busy_frac": avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simds / (us * 1e3 * clock_ghz),
           "wave_cycle_split": {k: avg[c] / avg["SQ_WAVE_CYCLES"] for k, c in
                                (("waiting", "SQ_WAIT_ANY"), ("issue_stalled", "SQ_WAIT_INST_ANY"),
                                 ("issuing", "SQ_ACTIVE_INST_ANY"), ("valu", "SQ_ACTIVE_INST_VALU"))}}
    return out


def main():
    res = {f: summarize(f) for f in (sys.argv[2:] or ["x3", "f32"])}
    json.dump(res, open(sys.argv[1], "w"), indent=1)
    for f, r in res.items():
        if r:
            print(f, r["kernel"], f"{r['kernel_us_profiled_median']:.0f} us", f"clock {r['clock_GHz']:.2f} GHz",
                  f"matrix pipe {r['matrix_pipe_busy_frac']:.2f}", {k: round(v, 3) for k, v in r["wave_cycle_split"].items()})


if __name__ == "__main__":
    main()
