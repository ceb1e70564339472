#!/usr/bin/env python3
"""Diagnostic (not product): can two RCCL ranks share ONE GPU on this pool's one-GPU boxes? If so,
bench.py's multi-rank path (QUAD_BENCH_REHEARSAL=nccl) can be rehearsed over RCCL itself rather
than gloo. Starts 2 ranks (subprocesses, 127.0.0.1 rendezvous), both on cuda:0, and runs one
all_reduce(SUM) of a 37,001-float bucket (the PPO gradient bucket's size) plus a barrier.

    python tools/diag/rccl_same_gpu.py
"""
import os
import subprocess
import sys
import time


def rank_main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((37001,), float(rank + 1), device="cuda:0")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    ok = bool((t == sum(range(1, world + 1))).all())
    ts = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_reduce(t)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    dist.barrier()
    print(f"rank {rank}: all_reduce ok={ok}, median {sorted(ts)[len(ts) // 2]:.1f} us (2 ranks on one GPU)", flush=True)
    dist.destroy_process_group()


def main():
    if "RANK" in os.environ:
        return rank_main()
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)],
                              env=dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
             for r in range(2)]
    rcs = [p.wait(timeout=240) for p in procs]
    print("exit codes", rcs)
    sys.exit(max(abs(r) for r in rcs))


if __name__ == "__main__":
    main()
