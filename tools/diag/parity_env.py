"""Diagnostic (not product): per-field error of one env of test_step_matches_oracle_random_states."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_parity as T
from oracle import oracle as O
n = 3000; kind = wrap = 0
rng = np.random.default_rng(17 + kind * 2 + wrap)
st = T._random_states(n, rng)
acts = rng.uniform(-1.3, 1.3, (n, 4)).astype(np.float32)
env = T._env(n, "hover", None, auto_reset=False)
g = T._gpu_step(env, st, acts)
ref = T._oracle_step(kind, wrap, st, acts)
worst = []
for i, o in enumerate(ref):
    for f, pre in (("qpos", st["qpos"][i]), ("qvel", st["qvel"][i]), ("obs", None), ("reward", None), ("state12", None)):
        gv = np.atleast_1d(np.asarray(g[f][i], np.float64)); rv = np.atleast_1d(np.asarray(o[f], np.float64))
        sc = np.abs(rv) if pre is None else np.maximum(np.abs(rv), np.abs(pre))
        r = np.abs(gv - rv) / (1e-5 * sc + 1e-6)
        j = int(np.argmax(r)); worst.append((r[j], i, f, j, gv[j], rv[j], (pre[j] if pre is not None else None)))
worst.sort(reverse=True)
for w in worst[:8]:
    print("ratio %.3f env %d %s[%d] got %.9g ref %.9g pre %s" % w)
print("state of worst:", {k: st[k][worst[0][1]] for k in ("qpos", "qvel")}, "act", acts[worst[0][1]])
