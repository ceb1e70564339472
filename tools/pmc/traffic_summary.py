#!/usr/bin/env python3
"""Profiling tool (not product): summarize tools/pmc/traffic_round.sh's rocprofv3 CSVs into
profiles/<round>/pmc_traffic.json and profiles/pmc_traffic.json (read by bench.py), keyed by the
step kernel's template symbol as rocprofv3 names it (e.g. "k_step_h<0, false, true, 256>") and then
by the env count, so the bench attaches a figure only to the kernel it actually timed.

Method (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE (KiB) come from separate
passes (3 + 2 TCC slots); they derive from the L2's memory-side request counters (Infinity-Cache
hits are counted, not excluded), FETCH_SIZE under-reads wide streaming loads by 2x and other access
widths are uncalibrated -> every figure is scaled by the factor measured on tools/pmc/pmc_calib.hip
(a dword-per-lane coalesced copy: the step kernels' SoA access shape) over a known byte count.
Per launch = the median over the profiled launches. Durations from the kernel-trace pass of the
same driver (tools/step_once.py: eager launches, random actions, auto-reset on).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

BYTES_PER_ENV_STEP = 278   # state r/w 2 x 104, action 16, obs 48 + reward 4 + flags 2
READ_PER_ENV_STEP = 120    # state 104 + action 16
WRITE_PER_ENV_STEP = 158   # state 104 + obs 48 + reward 4 + flags 2


def symbol(kernel_name: str) -> str:
    """'void (anonymous namespace)::k_step_h<0, false, true, 256>(float*, ...)' -> 'k_step_h<0, false, true, 256>'"""
    m = re.search(r"(k_step\w*<[^>]*>)", kernel_name)
    return m.group(1) if m else kernel_name


def per_kernel(pattern, counter):
    d = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                d.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return d


def trace_avg(root, n):
    out = {}
    for f in glob.glob(f"{root}/trace_{n}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_step" in r["Name"]:
                out[symbol(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                          "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    return out


def main(root, out_dirs, round_tag):
    cal_f = per_kernel(f"{root}/cal_fetch/**/*counter_collection.csv", "FETCH_SIZE")
    cal_w = per_kernel(f"{root}/cal_write/**/*counter_collection.csv", "WRITE_SIZE")
    calib_bytes = float(os.environ.get("CALIB_BYTES", 4 * (64 << 20)))
    kf = [statistics.median(v) for k, v in cal_f.items() if "calib" in k]
    kw = [statistics.median(v) for k, v in cal_w.items() if "calib" in k]
    f_scale = calib_bytes / (kf[0] * 1024)
    w_scale = calib_bytes / (kw[0] * 1024)
    res = {"method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over tools/step_once.py "
                     "(eager quad_step launches, random actions, auto-reset on); KiB x 1024 x the calibration "
                     "scale of a dword-per-lane coalesced copy of known size (tools/pmc/pmc_calib.hip); median "
                     "per launch. L2 memory-side bytes: Infinity-Cache hits are included (no MALL counter on "
                     "gfx950 separates them), so only the sizes past the 256 MiB cache are DRAM-bound.",
           "round": round_tag,
           "calibration": {"pattern": "dword-per-lane coalesced copy", "bytes": calib_bytes,
                           "fetch_scale": f_scale, "write_scale": w_scale},
           "kernels": {}}
    for path in sorted(glob.glob(f"{root}/fetch_*")):
        if not os.path.isdir(path):
            continue
        n = int(path.rsplit("_", 1)[1])
        fetch = per_kernel(f"{path}/**/*counter_collection.csv", "FETCH_SIZE")
        write = per_kernel(f"{root}/write_{n}/**/*counter_collection.csv", "WRITE_SIZE")
        traces = trace_avg(root, n)
        for name, v in fetch.items():
            if "k_step" not in name:
                continue
            sym = symbol(name)
            fb = statistics.median(v) * 1024 * f_scale
            wb = statistics.median(write.get(name, [0.0])) * 1024 * w_scale
            alg = BYTES_PER_ENV_STEP * n
            rec = {"kernel": name, "envs": n, "launches_profiled": len(v),
                   "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                   "algorithmic_bytes": alg, "traffic_over_algorithmic": (fb + wb) / alg,
                   "fetch_over_algorithmic_reads": fb / (READ_PER_ENV_STEP * n),
                   "write_over_algorithmic_writes": wb / (WRITE_PER_ENV_STEP * n),
                   "raw_FETCH_SIZE_KiB": statistics.median(v),
                   "raw_WRITE_SIZE_KiB": statistics.median(write.get(name, [0.0])),
                   "working_set_vs_infinity_cache": "inside (256 MiB)" if (fb + wb) < 200e6 else
                   ("straddles" if (fb + wb) < 400e6 else "outside: DRAM-bound")}
            if sym in traces:
                t = traces[sym]
                rec["trace_avg_ns"] = t["avg_ns"]
                rec["traffic_GBs_at_trace_avg"] = (fb + wb) / t["avg_ns"]
                rec["algorithmic_GBs_at_trace_avg"] = alg / t["avg_ns"]
            res["kernels"].setdefault(sym, {})[str(n)] = rec
    for d in out_dirs:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "pmc_traffic.json"), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3:], sys.argv[2])
