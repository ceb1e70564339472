#!/usr/bin/env python3
"""Diagnostic (not product): would the rollout critic's layer 2 hold test_gpu_policy's bar
|d| <= 2e-5 (1 + |ref|) on fewer bf16 pieces? (option A.) NumPy emulation of the
split products of policy_net.h: every f32 operand x = p0 + p1 (+ p2), each piece the round-to-nearest
bf16 of what the previous pieces leave, and the kept piece products summed exactly (float64: the MFMA's
f32 accumulation only adds rounding). SB3-style orthogonal init (gain sqrt 2, value head gain 1), W2
perturbed and the value head scaled x30 to stand in for a trained critic (returns of O(10-100)).
Usage: critic_split_emu.py [n_rows]"""
import sys

import numpy as np


def bf16(x):
    b = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return (((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16).astype(np.uint32).view(np.float32)


def pieces(x, n):
    out, r = [], x.astype(np.float32)
    for _ in range(n):
        p = bf16(r)
        out.append(p)
        r = (r - p).astype(np.float32)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    rng = np.random.default_rng(0)

    def orth(r, c, gain):
        q, _ = np.linalg.qr(rng.standard_normal((max(r, c), max(r, c))))
        return (gain * q[:r, :c]).astype(np.float32)

    W1, b1 = orth(128, 12, np.sqrt(2)), (rng.standard_normal(128) * 0.05).astype(np.float32)
    W2, b2 = orth(128, 128, np.sqrt(2)), (rng.standard_normal(128) * 0.05).astype(np.float32)
    W2 = (W2 + rng.standard_normal(W2.shape).astype(np.float32) * 0.05).astype(np.float32)
    W3, b3 = (orth(1, 128, 1.0) * 30).astype(np.float32), np.float32(0.1)
    x = rng.uniform(-1, 1, (n, 12)).astype(np.float32)
    h1 = np.maximum(x.astype(np.float64) @ W1.T.astype(np.float64) + b1, 0).astype(np.float32)
    h2_ref = np.maximum(h1.astype(np.float64) @ W2.T.astype(np.float64) + b2, 0)
    v_ref = h2_ref @ W3.T.astype(np.float64) + b3
    # (pieces of W2, pieces of h1, kept products a_i b_j): the product forms of 6, 5 and 3 MFMAs
    forms = [("3 x 3 pieces, 6 MFMAs (the product)", 3, 3, lambda i, j: i + j <= 2),
             ("3 x 2 pieces, 5 MFMAs", 3, 2, lambda i, j: i + j <= 2),
             ("2 x 2 pieces, 3 MFMAs (option A)", 2, 2, lambda i, j: i + j <= 1)]
    print(f"{n} rows, critic 12-128-128-1; error = |v - v_ref| / (1 + |v_ref|), bar 2e-5; mean |v_ref| {np.abs(v_ref).mean():.3g}")
    for name, na, nb, keep in forms:
        A, B = pieces(W2, na), pieces(h1, nb)
        acc = np.zeros((n, 128))
        for i in range(na):
            for j in range(nb):
                if keep(i, j):
                    acc += B[j].astype(np.float64) @ A[i].T.astype(np.float64)
        v = np.maximum(acc + b2, 0) @ W3.T.astype(np.float64) + b3
        e = np.abs(v - v_ref) / (1 + np.abs(v_ref))
        print(f"  {name:40s} max {e.max():.3g}  p99.99 {np.quantile(e, 0.9999):.3g}  {'holds' if e.max() <= 2e-5 else 'FAILS'} the bar")


if __name__ == "__main__":
    main()
