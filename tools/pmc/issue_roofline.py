#!/usr/bin/env python3
"""Summarize tools/pmc/issue_roofline.sh into profiles/<round>/pmc_issue.json and
profiles/pmc_issue.json (bench.py reads the latter into roofline.issue), keyed by the kernel's
template symbol and the env count: {"round": ..., "kernels": {symbol: {envs: record}}}, so the
bench attaches a record only to the kernel it timed.

Per step-kernel dispatch (median over dispatches 20..end, past the post-reset transient):
  instructions per 64 env-steps by class (SQ_INSTS_* / (envs / 64)): one step wave of 64 envs,
  plus -- in the helper-wave forms (k_step_h) -- the helper wave that shares its SIMD;
  the per-SIMD issue floor: a SIMD issues at most one wave64 vector instruction per 4 cycles
  (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), so the SIMD that holds those waves needs
  >= 4 * (VALU + VMEM + LDS) cycles + SALU/SMEM/branch slots;
  wave cycles and their split (SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY,
  quad-cycles), VALU-active share, and the effective clock GRBM_GUI_ACTIVE / 8 / kernel time."""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict


def load(root):
    d = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [values in dispatch order]
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(f)))
        rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)) or 0))
        for r in rows:
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            m = re.search(r"k_\w+<[^>]*>", r["Kernel_Name"])
            d[(m.group(0) if m else r["Kernel_Name"], grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def trace_us(root):
    out = {}
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        ks = [r for r in rows if "k_step" in r["Kernel_Name"]]
        if ks:
            du = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks[20:]] or \
                 [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
            out[int(ks[0].get("Grid_Size", ks[0].get("Grid_Size_X", 0)))] = statistics.median(du)
    return out


def main(root="gpurun_out/issue", rnd="r04"):
    res = {}
    sizes = sorted(int(m.group(1)) for m in (re.match(r"n(\d+)$", x) for x in os.listdir(root)) if m)
    for n in sizes:
        d = load(os.path.join(root, f"n{n}"))
        if not d:
            continue
        key = max(d, key=lambda k: len(d[k]))
        c = {k: statistics.median(v[20:] or v) for k, v in d[key].items()}
        waves = c.get("SQ_WAVES", 0) or 1
        units = n / 64  # SIMD slots: one step wave (+ its helper wave) per 64 envs
        per_wave = {k[len("SQ_INSTS_"):].lower(): c[k] / units for k in c if k.startswith("SQ_INSTS_")}
        vec = per_wave.get("valu", 0) + per_wave.get("vmem_rd", 0) + per_wave.get("vmem_wr", 0) + per_wave.get("lds", 0)
        sca = per_wave.get("salu", 0) + per_wave.get("smem", 0) + per_wave.get("branch", 0)
        t = trace_us(os.path.join(root, f"trace_{n}"))
        us = list(t.values())[0] if t else None
        r = {"grid": key[1], "envs": n, "waves": waves, "waves_per_64_envs": waves / units,
             "instructions_per_64_env_steps": per_wave, "vector_instructions_per_64_env_steps": vec,
             "scalar_instructions_per_64_env_steps": sca, "kernel_us_rocprof_trace": us}
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"] * 4 / waves  # quad-cycles -> cycles, mean wave lifetime
            r["wave_cycles"] = wc
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
                if k in c:
                    r[k.lower() + "_share"] = c[k] * 4 / waves / wc
            # per-SIMD issue floor vs the measured wave lifetime (same counters, same dispatches)
            r["issue_floor_cycles"] = 4 * vec + sca
            r["frac_issue_floor"] = r["issue_floor_cycles"] / wc
        if us and "GRBM_GUI_ACTIVE" in c:
            # GRBM_GUI_ACTIVE per XCD over the traced kernel time; above the 2.4 GHz peak clock it
            # holds profiler serialization around a short dispatch and is not a clock
            clk = c["GRBM_GUI_ACTIVE"] / 8 / (us * 1e3)
            if clk <= 2.5:
                r["effective_clock_GHz"] = clk
        res.setdefault(key[0], {})[str(n)] = r
    out = {"round": rnd, "source": "tools/pmc/issue_roofline.sh (rocprofv3 PMC over tools/step_once.py)",
           "kernels": res}
    for d in (os.path.join("profiles", rnd), "profiles"):
        os.makedirs(d, exist_ok=True)
        json.dump(out, open(os.path.join(d, "pmc_issue.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
