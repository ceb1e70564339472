"""bench.py at world > 1 (config 4: 524,288 hover envs over 8 GPUs, one RCCL gradient all-reduce per
optimizer step; reference train_brax_ppo.py:589-620 pmean of grads): what its line must carry so
that the driver's first 8-GPU run is verifiable, rehearsed with 2 gloo ranks on one GPU
(QUAD_BENCH_REHEARSAL=1) at a small size:
  * end_to_end.n_ranks as torch.distributed sees them;
  * end_to_end.allreduce: every gradient all-reduce of the timed update HIP-event timed around the
    collective and work.wait(), its share of the optimizer step, and the collective alone;
  * end_to_end.shard_identity: each rank's step digest equals the same global ids' rows of one
    handle of all the ranks' envs;
  * the episode statistics of a rollout reduced over the ranks, equal to one process
    stepping every rank's envs;
  * per_rank / end_to_end.per_rank: every rank's elapsed, kernel and all-reduce figures with
    min / max / argmax rank (skew is visible, not hidden in the MAX over ranks).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (the rank-0-only configs run too: nothing rank 0 does alone may join a collective)
SMALL = ["--steps", "20", "--warmup", "5", "--graph-chunk", "10", "--kernel-launches", "20",
         "--large-envs", "0", "--dram-envs", "0", "--rollout-steps", "0",
         "--no-cpu-baseline", "--e2e-iters", "1", "--e2e-steps", "16", "--e2e-epochs", "1"]


def _run(gpus: int, envs: int, rehearsal: bool) -> dict:
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        e.pop(k, None)
    if rehearsal:
        e["QUAD_BENCH_REHEARSAL"] = "1"
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", str(gpus),
                        "--envs", str(envs)] + SMALL, env=e, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_two_rank_bench_line_is_verifiable():
    n = 4096
    two = _run(2, n, rehearsal=True)
    one = _run(1, 2 * n, rehearsal=False)
    e2, e1 = two["end_to_end"], one["end_to_end"]
    assert two["n_gpus"] == 2 and e2["n_ranks"] == 2 and e2["world_size"] == 2 and e1["n_ranks"] == 1
    assert e2["global_envs"] == e1["global_envs"] == 2 * n
    # (a) the gradient all-reduce of every optimizer step of the timed update, timed on its stream
    ar = e2["allreduce"]
    assert ar["count"] == e2["n_epochs"] * e2["minibatches_per_epoch"] * e2["iterations"]
    assert 0.0 < ar["median_us"] <= ar["max_us"] and ar["mean_us"] > 0.0
    # a wall-time ratio (two ranks share one GPU here): reported, finite and positive, not a bar
    assert 0.0 < ar["exposed_share_of_optimizer_step"] < float("inf")
    assert ar["backend"] == "gloo" and ar["alone"]["bytes"] == 37001 * 4 and ar["alone"]["us_per_allreduce"] > 0.0
    assert "allreduce" not in e1
    # (d) per-rank figures: a slow GPU or link must be visible, not only the MAX over ranks
    pr = two["per_rank"]
    assert [r["rank"] for r in pr["ranks"]] == [0, 1]
    for k in ("elapsed_s", "region_us", "kernel_us"):
        assert 0.0 < pr[k]["min"] <= pr[k]["max"] and pr[k]["argmax_rank"] in (0, 1), k
        assert [r[k] for r in pr["ranks"]][pr[k]["argmax_rank"]] == pr[k]["max"], k
    assert pr["elapsed_s"]["max"] == pytest.approx(two["ms_per_step"] * two["steps"] / 1e3, rel=1e-9)
    epr = e2["per_rank"]
    for k in ("wall_s", "train_s", "allreduce_median_us", "allreduce_max_us"):
        assert 0.0 < epr[k]["min"] <= epr[k]["max"], k
    assert all(r["allreduce_median_us"] > 0.0 for r in epr["ranks"])
    assert "per_rank" not in one and "per_rank" not in e1
    assert "config1_train_py_on_gpu" in one["configs"] and "config1_train_py_on_gpu" not in two["configs"]
    # (b) each rank's shard is the same bits as those global ids in one handle
    si = e2["shard_identity"]
    assert si["all_equal"] and len(si["rank_digests"]) == 2 and si["one_handle_envs"] == 2 * n
    assert si["rank_digests"][0] != si["rank_digests"][1]
    # (c) the first rollout's episode statistics reduced over the ranks == one process over all envs
    p2, p1 = e2["episodes_first_rollout"], e1["episodes_first_rollout"]
    assert p2["reduced_over_ranks"] and not p1["reduced_over_ranks"]
    assert p2["count"] == p1["count"] > p2["local_count"] > 0
    for k in ("return_sum", "length_sum"):
        assert p2[k] == pytest.approx(p1[k], rel=1e-12), k
