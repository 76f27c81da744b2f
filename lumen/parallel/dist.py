"""Process-group setup: one process per GPU, RCCL (``backend="nccl"`` on ROCm) or gloo on CPU.

Reference behaviour: DeepSpeed/accelerate init (reference training/train.ipynb:780-806) reading
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the launcher, world = one DP group.
Fixes reference quirk 12: the visible-device set is never widened -- a rank whose
LOCAL_RANK exceeds the visible devices fails with a clear message before any RCCL call instead
of `invalid device ordinal` (training/train.ipynb:806).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_ENV: Optional[DistEnv] = None


def env_ints():
    g = os.environ.get
    world = int(g("WORLD_SIZE", g("SLURM_NTASKS", "1")))
    rank = int(g("RANK", g("SLURM_PROCID", "0")))
    local = int(g("LOCAL_RANK", g("SLURM_LOCALID", "0")))
    local_world = int(g("LOCAL_WORLD_SIZE", str(world)))
    return rank, world, local, local_world


def init(backend: Optional[str] = None, device: Optional[str] = None,
         timeout_s: Optional[int] = None) -> DistEnv:
    """Initialise (idempotent).  backend None -> 'nccl' (RCCL) when GPUs are visible, else gloo.

    A hung collective fails after ``LUMEN_DIST_TIMEOUT`` seconds (default 1800) with async error
    handling on, so a dead peer ends the job instead of stalling it."""
    global _ENV
    if _ENV is not None:
        return _ENV
    from ..utils.debug import apply_debug_env

    apply_debug_env()  # before the first HIP call
    if timeout_s is None:
        timeout_s = int(os.environ.get("LUMEN_DIST_TIMEOUT", "1800"))
    rank, world, local, local_world = env_ints()
    want_gpu = device != "cpu" and (device == "cuda" or torch.cuda.is_available())
    shared = os.environ.get("LUMEN_SHARED_GPU_REHEARSAL", "0") == "1" and world > 1
    if want_gpu:
        ndev = torch.cuda.device_count()
        if shared:
            # rehearsal of the multi-rank RCCL path on fewer GPUs than ranks (testing only):
            # ranks share devices round-robin, and each rank claims its own RCCL "host" so
            # RCCL's duplicate-device check passes and the ranks talk over its socket transport
            # (loopback).  Collective semantics are RCCL's; timings mean nothing.
            os.environ["NCCL_HOSTID"] = f"lumen-rehearsal-{rank}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            local = local % max(ndev, 1)
        elif local >= ndev:
            raise RuntimeError(
                f"LOCAL_RANK={local} but only {ndev} GPU(s) are visible "
                f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')}, "
                f"ROCR_VISIBLE_DEVICES={os.environ.get('ROCR_VISIBLE_DEVICES')}); "
                "launch at most one rank per visible GPU")
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if backend is None:
        backend = "nccl" if dev.type == "cuda" else "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
        if backend == "nccl":
            # the host-side gloo group, created here where every rank is at the same point
            # (new_group is collective): later first uses cannot be reached in different orders
            host_group()
    _ENV = DistEnv(rank, world, local, local_world, backend if world > 1 else "none", dev)
    return _ENV


def get_env() -> DistEnv:
    return _ENV if _ENV is not None else init()


def barrier():
    if dist.is_initialized():
        e = get_env()
        if e.backend == "nccl":
            dist.barrier(device_ids=[e.device.index])
        else:
            dist.barrier()


def all_reduce_scalar(x: float, op=dist.ReduceOp.SUM) -> float:
    if not dist.is_initialized():
        return x
    e = get_env()
    t = torch.tensor([x], dtype=torch.float64 if e.device.type == "cpu" else torch.float32,
                     device=e.device)
    dist.all_reduce(t, op=op)
    return float(t.item())


_HOST_GROUP = None


def host_group():
    """A gloo group over every rank for host-side agreements (values the host already holds,
    e.g. a per-step scheduling decision): no device work, no stream sync.  On a gloo world this
    is the default group (None).  ``init`` creates it right after the process group (every rank
    at the same point: ``new_group`` is collective)."""
    global _HOST_GROUP
    if not dist.is_initialized() or dist.get_backend() == "gloo":
        return None
    if _HOST_GROUP is None:
        _HOST_GROUP = dist.new_group(backend="gloo")
    return _HOST_GROUP


def agree_all(flag: bool) -> bool:
    """True only if ``flag`` is True on every rank (MIN all-reduce on the host group)."""
    if not dist.is_initialized():
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=host_group())
    return bool(t.item())


def broadcast_object(obj, src: int = 0):
    if not dist.is_initialized():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def shutdown():
    global _ENV, _HOST_GROUP
    if dist.is_initialized():
        try:
            barrier()
        finally:
            dist.destroy_process_group()
    _ENV = None
    _HOST_GROUP = None
