#!/usr/bin/env python3
"""Profiling tool (not product): per-burst duration summary of one kernel in a rocprofv3
--kernel-trace CSV, so the bench's timed region (graph-replayed, back-to-back launches) can be
compared with its HIP-event figure apart from warmup and single-launch measurements.
Usage: trace_bursts.py TRACE.csv KERNEL_SUBSTRING GRID [MIN_LAUNCHES]"""
import csv
import sys


def main():
    path, name, grid = sys.argv[1], sys.argv[2], int(sys.argv[3])
    min_n = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    rows = [r for r in csv.DictReader(open(path))
            if name in r["Kernel_Name"] and int(r.get("Grid_Size", r.get("Grid_Size_X", 0))) == grid]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    bursts, cur = [], [0]
    for i in range(1, len(rows)):  # a burst: launches starting < 50 us after the previous one
        if st[i] - st[i - 1] < 50_000:
            cur.append(i)
        else:
            bursts.append(cur)
            cur = [i]
    bursts.append(cur)
    print(f"kernel ~ {name!r}, grid {grid}: {len(rows)} launches, bursts of >= {min_n}:")
    for b in bursts:
        if len(b) < min_n:
            continue
        d = sorted((en[i] - st[i]) / 1e3 for i in b)
        wall = (en[b[-1]] - st[b[0]]) / 1e3 / len(b)
        print(f"  {len(b):5d} launches: mean {sum(d) / len(d):.3f} us, median {d[len(d) // 2]:.3f} us, "
              f"wall per launch {wall:.3f} us")


if __name__ == "__main__":
    main()
