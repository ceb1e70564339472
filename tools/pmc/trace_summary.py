#!/usr/bin/env python3
"""Per-kernel, per-grid-size duration summary of a rocprofv3 --kernel-trace CSV."""
import csv
import sys
from collections import defaultdict

def short(name):
    """Drop the trailing argument list: cut at the '(' that opens the last top-level group."""
    depth = 0
    for i in range(len(name) - 1, -1, -1):
        if name[i] == ")":
            depth += 1
        elif name[i] == "(":
            depth -= 1
            if depth == 0:
                return name[:i].replace("void ", "").replace("(anonymous namespace)::", "")
    return name


rows = list(csv.DictReader(open(sys.argv[1])))
d = defaultdict(list)
for r in rows:
    d[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = ["kernel,grid_threads,calls,mean_us,median_us,min_us,max_us,vgpr"]
vg = {(short(r["Kernel_Name"]), int(r["Grid_Size_X"])): r["VGPR_Count"] for r in rows}
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    out.append(f"{k[0]},{k[1]},{len(v)},{sum(v)/len(v):.3f},{v[len(v)//2]:.3f},{v[0]:.3f},{v[-1]:.3f},{vg[k]}")
print("\n".join(out))
