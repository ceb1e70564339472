"""bench.py's rank launch (the contract's `--gpus N`): no GPU needed.

`--check-launch` runs only the rank topology on gloo, so these tests cover both ways the driver
can start N ranks -- bench.py's own launcher (`--gpus N`, one child per GPU) and
`torch.distributed.run --nproc-per-node N` -- and that the reported n_gpus / global_envs follow N.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        e.pop(k, None)
    return e


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 4])
def test_gpus_flag_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--check-launch"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    d = _last_json(r.stdout)
    assert d["n_gpus"] == n
    assert d["global_envs"] == n * 65536
    assert d["ranks_sum"] == n * (n - 1) / 2


def test_torchrun_launch_matches_gpus_flag():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2",
                        "--check-launch"], env=_env(), capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode == 0, r.stderr
    assert _last_json(r.stdout)["n_gpus"] == 2


def test_world_size_mismatch_is_refused():
    e = _env()
    e.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--check-launch"], env=e,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "--gpus 1" in r.stderr


def test_launch_terms_arithmetic():
    """roofline.frac_beyond_launch_floor / frac_ceiling_one_launch (bench.py _launch_terms): the
    HBM fraction of the time past the dispatch floor, and what a zero-latency one-launch step of the
    same bytes could reach -- 18.2 MB at 8 TB/s = 2.28 us beside a 1.62 us floor caps it at 0.58."""
    sys.path.insert(0, REPO)
    import bench
    byt = bench.BYTES_PER_ENV_STEP * 65536
    at_peak_us = byt / (bench.HBM_PEAK_GBS * 1e3)
    d = bench._launch_terms({"launch_floor_us": 1.62, "kernel_us": 5.94}, 65536)
    assert d["launch_floor_us"] == 1.62
    assert abs(d["frac_ceiling_one_launch"] - at_peak_us / (at_peak_us + 1.62)) < 1e-12
    assert 0.58 < d["frac_ceiling_one_launch"] < 0.59
    assert abs(d["frac_beyond_launch_floor"] - at_peak_us / (5.94 - 1.62)) < 1e-12
    # no floor measured (or a kernel faster than it): no derived fields, never a division by <= 0
    assert bench._launch_terms({"kernel_us": 5.94}, 65536) == {}
    assert bench._launch_terms({"launch_floor_us": 2.0, "kernel_us": 1.5}, 65536)["frac_beyond_launch_floor"] is None
