#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSVs (FETCH_SIZE pass, WRITE_SIZE pass, calibration) into
profiles/<round>/pmc_quad_step.json and profiles/pmc_quad_step.json (read by bench.py).

gfx950 (MI355X_MICROARCH.md, HBM): FETCH_SIZE / WRITE_SIZE are in KiB and derive from the L2's
memory-side request counters; FETCH_SIZE under-reads wide streaming loads by 2x and other
widths are uncalibrated -> every figure here is scaled by the factor measured on
tools/pmc/pmc_calib.hip (a dword-per-lane coalesced copy, k_step's access shape) with a known
byte count.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pattern):
    rows = []
    for f in glob.glob(pattern, recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def per_kernel(rows, counter):
    d = defaultdict(list)
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        d[(r["Kernel_Name"], grid)].append(float(r["Counter_Value"]))
    return d


def main(root, out_dirs):
    fetch = per_kernel(load(f"{root}/pmc_fetch/**/*counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(load(f"{root}/pmc_write/**/*counter_collection.csv"), "WRITE_SIZE")
    cal_f = per_kernel(load(f"{root}/pmc_cal_fetch/**/*counter_collection.csv"), "FETCH_SIZE")
    cal_w = per_kernel(load(f"{root}/pmc_cal_write/**/*counter_collection.csv"), "WRITE_SIZE")
    calib_bytes = float(os.environ.get("CALIB_BYTES", 4 * (64 << 20)))

    def med(v):
        v = sorted(v)
        return v[len(v) // 2]
    kf = [med(v) for k, v in cal_f.items() if "calib" in k[0]]
    kw = [med(v) for k, v in cal_w.items() if "calib" in k[0]]
    f_scale = calib_bytes / (kf[0] * 1024) if kf else 2.0
    w_scale = calib_bytes / (kw[0] * 1024) if kw else 1.0
    res = {"calibration": {"pattern": "dword-per-lane coalesced copy", "bytes": calib_bytes,
                           "fetch_scale": f_scale, "write_scale": w_scale}}
    for (name, grid), v in fetch.items():
        if "k_step" not in name:
            continue
        wv = write.get((name, grid), [0.0])
        fb = med(v) * 1024 * f_scale
        wb = med(wv) * 1024 * w_scale
        res[str(grid)] = {"kernel": name, "fetch_bytes": fb, "write_bytes": wb,
                          "hbm_bytes_per_launch": fb + wb, "algorithmic_bytes": 278 * grid,
                          "traffic_over_algorithmic": (fb + wb) / (278 * grid),
                          "raw_FETCH_SIZE_KiB": med(v), "raw_WRITE_SIZE_KiB": med(wv)}
    for d in out_dirs:
        os.makedirs(d, exist_ok=True)
        json.dump(res, open(os.path.join(d, "pmc_quad_step.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
