#!/usr/bin/env python3
"""Static instruction histogram of one kernel in a device assembly file (hipcc --cuda-device-only -S).

    python tools/isa/isa_hist.py quadenv.s k_stepILi0ELb0E [--blocks]

Counts opcodes per class (f32 VALU, f64 VALU, other VALU, SALU, VMEM, LDS, branch/wait) over the
kernel body; with --blocks, per basic block (label) so the straight-line step can be told apart
from the reset / bad-state branches."""
import re
import sys
from collections import Counter, OrderedDict


def body(lines, key):
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(key) + r"\w*:", l))
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end") or re.match(r"^\s*\.size", l):
            break
        out.append(l)
    return out


def klass(op):
    if op.startswith("v_"):
        if "_f64" in op or op.startswith("v_fma_f64") or "f64" in op:
            return "valu_f64"
        if op.startswith(("v_mfma", "v_smfma")):
            return "mfma"
        if "_f32" in op or "f32" in op:
            return "valu_f32"
        return "valu_other"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_barrier", "s_nop", "s_endpgm", "s_setprio",
                      "s_sleep")):
        return "control"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, key = sys.argv[1], sys.argv[2]
    per_block = "--blocks" in sys.argv
    lines = open(path).read().splitlines()
    b = body(lines, key)
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for l in b:
        m = re.match(r"^(\.LBB\w+|\w+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        blocks[cur].append(t.split()[0])
    total = Counter()
    for name, ops in blocks.items():
        c = Counter(klass(o) for o in ops)
        total.update(c)
        if per_block and ops:
            print(f"{name:>14} {len(ops):5d}  " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
    allops = Counter(o for ops in blocks.values() for o in ops)
    print("total", sum(total.values()), dict(sorted(total.items())))
    print("top:", ", ".join(f"{o}={n}" for o, n in allops.most_common(40)))


if __name__ == "__main__":
    main()
