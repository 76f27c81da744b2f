"""Multi-rank RCCL semantics probe (run under torch.distributed.run, any world size).

Initialises through ``lumen.parallel.dist.init`` (so LUMEN_SHARED_GPU_REHEARSAL works) and checks
the collectives the training and serving paths issue against values every rank can compute:
all_reduce (sum, max), all_gather_into_tensor, reduce_scatter_tensor, broadcast, a split
communicator (``new_group``) and the coalesced bucket sizes lumen's ZeRO code uses.  Prints one
``rccl_probe ok`` line per rank, or raises.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import torch.distributed as dist

    from lumen.parallel.dist import barrier, init, shutdown

    env = init()
    r, W, dev = env.rank, env.world_size, env.device
    assert env.backend == "nccl", env.backend
    # all_reduce sum / max
    x = torch.full((1 << 20,), float(r + 1), device=dev)
    dist.all_reduce(x)
    assert torch.all(x == W * (W + 1) / 2), x[:4]
    m = torch.tensor([float(r)], device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    assert m.item() == W - 1
    # all_gather_into_tensor (ZeRO-3 unit gather shape: bf16 shards)
    n = 386 * (1 << 20) // 2 // W  # one 7B decoder layer's shard, bf16
    shard = torch.full((n,), float(r), device=dev, dtype=torch.bfloat16)
    full = torch.empty(n * W, device=dev, dtype=torch.bfloat16)
    dist.all_gather_into_tensor(full, shard)
    ref = torch.arange(W, device=dev, dtype=torch.bfloat16).repeat_interleave(n)
    assert torch.equal(full, ref)
    # reduce_scatter_tensor (ZeRO-2/3 gradient bucket: 2e6 f32 elements)
    b = 2_000_000 // W * W
    g = torch.arange(b, device=dev, dtype=torch.float32) + r
    out = torch.empty(b // W, device=dev)
    dist.reduce_scatter_tensor(out, g)
    lo = r * (b // W)
    exp = (torch.arange(lo, lo + b // W, device=dev, dtype=torch.float32) * W
           + W * (W - 1) / 2)
    assert torch.allclose(out, exp), (out[:4], exp[:4])
    # broadcast from the last rank
    t = torch.full((4096,), float(r), device=dev)
    dist.broadcast(t, src=W - 1)
    assert torch.all(t == W - 1)
    # split communicator (the ZeRO-3 gather group when LUMEN_ZERO3_SHARED_GROUP is unset)
    grp = dist.new_group(list(range(W)))
    y = torch.ones(1024, device=dev)
    dist.all_reduce(y, group=grp)
    assert torch.all(y == W)
    torch.cuda.synchronize()
    barrier()
    print(f"rccl_probe ok rank {r}/{W} device {dev} "
          f"NCCL_HOSTID={os.environ.get('NCCL_HOSTID')}", flush=True)
    shutdown()


if __name__ == "__main__":
    main()
