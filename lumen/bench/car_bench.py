"""Custom all-reduce latency sweep (lumen/parallel/custom_ar.py).

    python -m lumen.bench.car_bench [--world 2] [--out car_bench.json]

Without an 8-GPU node this runs ``world`` processes on ONE GPU: the IPC mapping and barrier
protocol are real, but every "peer" load stays on the device. The numbers therefore show
kernel and barrier overhead and the uncached-vs-cached staging trade-off, not xGMI
bandwidth. On a multi-GPU node, set ``LUMEN_CAR_BENCH_MULTI=1`` to give each rank its own GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import time


def _worker(rank, world, port, out, sizes, multi):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(rank if multi else 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lumen.parallel.custom_ar import CustomAllReduce

    dev = torch.device("cuda", torch.cuda.current_device())
    rows = []
    for cached in (False, True):
        car = CustomAllReduce(dist.group.WORLD, dev, max_bytes=max(sizes), cached=cached,
                              timeout_s=20.0)
        for nbytes in sizes:
            t = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=dev)
            for two in (False, True):
                for _ in range(10):
                    car.all_reduce(t, two_shot=two)
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                n = 100
                for _ in range(n):
                    car.all_reduce(t, two_shot=two)
                torch.cuda.synchronize()
                us = (time.perf_counter() - t0) / n * 1e6
                rows.append({"cached": cached, "bytes": nbytes, "two_shot": two, "us": us,
                             "plan": car.plan(nbytes, nbytes // 2)})
        car.check()
        dist.barrier()
        car.close()
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"world": world, "multi_gpu": multi, "rows": rows}, f, indent=1)
        for r in rows:
            print(f"cached={int(r['cached'])} {r['bytes'] >> 10:6d} KiB "
                  f"{'two' if r['two_shot'] else 'one'}-shot {r['us']:8.1f} us", flush=True)
    dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--out", default="car_bench.json")
    a = ap.parse_args()
    sizes = [8 << 10, 32 << 10, 128 << 10, 512 << 10, 2 << 20]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    multi = os.environ.get("LUMEN_CAR_BENCH_MULTI", "0") == "1"
    mp.spawn(_worker, args=(a.world, port, a.out, sizes, multi), nprocs=a.world, join=True)


if __name__ == "__main__":
    main()
