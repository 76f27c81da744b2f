"""Custom all-reduce over IPC-mapped peer memory for tensor-parallel decode.

The kernel is in ``lumen/csrc/kernels/custom_ar.hip``. It is a one-shot or two-shot reduction
through uncached staging buffers that every rank maps from every peer, with per-block
epoch barriers.

This class owns the buffers. Construction is collective over ``group``:

1. each rank allocates its staging buffer and its signal block;
2. the ranks exchange ``hipIpcMemHandle`` bytes with ``all_gather_object``;
3. each rank opens its peers' handles.

``group`` can be an RCCL or a gloo group; only the handle exchange uses it.

A call launches one kernel with fixed arguments: the peer pointer tables and the caller's
tensors. That makes it capturable in the hipGraph of a TP decode bucket, which RCCL is not.

Use ``eligible(t)`` to decide whether a tensor goes here or to RCCL. The tensor must be:

* at most ``max_bytes``;
* contiguous;
* ``numel % 8 == 0``;
* f32, f16 or bf16.

Messages up to ``one_shot_max`` bytes use one-shot (every rank reads all peers); larger ones
use two-shot (reduce-scatter then all-gather through the same buffers).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops._native import native

_DTYPES = (torch.float32, torch.float16, torch.bfloat16)


class CollectiveTimeout(RuntimeError):
    """A custom all-reduce / all-gather barrier gave up waiting for a peer."""


def _default_one_shot_max(world: int) -> int:
    # one-shot reads (W-1)·n over the links vs 2(W-1)/W·n for two-shot plus one more barrier;
    # the crossover moves down as W grows
    return {2: 1 << 20, 4: 512 << 10}.get(world, 256 << 10)


class CustomAllReduce:
    def __init__(self, group=None, device: Optional[torch.device] = None,
                 max_bytes: int = 8 << 20, one_shot_max: Optional[int] = None,
                 timeout_s: Optional[float] = None, cached: Optional[bool] = None):
        C = native()
        if C is None or not hasattr(C, "car_allreduce"):
            raise RuntimeError("lumen native extension with car_* ops is not built")
        self.C = C
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > C.car_max_ranks():
            raise ValueError(f"custom all-reduce supports up to {C.car_max_ranks()} ranks")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = int(max_bytes)
        self.one_shot_max = int(one_shot_max if one_shot_max is not None
                                else _default_one_shot_max(self.world))
        self.timeout_s = float(timeout_s if timeout_s is not None
                               else os.environ.get("LUMEN_CAR_TIMEOUT", "30"))
        self.max_blocks = C.car_max_blocks()
        # staging buffers: uncached by default (always coherent across devices); cached relies
        # on the barrier fences' L2 writeback/invalidate (LUMEN_CAR_CACHED=1)
        self.cached = bool(cached if cached is not None
                           else os.environ.get("LUMEN_CAR_CACHED", "0") == "1")
        # every step below is collective; a rank that fails still takes part in both
        # exchanges, so either all ranks end up with the custom path or all raise
        self._buf = self._sig = None
        self._flag_host = self._flag_dev = 0
        self._opened: List[int] = []
        self.data: List[int] = []
        self.sig: List[int] = []
        err = None
        with torch.cuda.device(self.device):
            mine = None
            try:
                self._buf = C.car_alloc(self.max_bytes, self.cached)
                self._sig = C.car_alloc(C.car_signal_bytes(), False)
                mine = (C.car_handle(self._buf), C.car_handle(self._sig))
            except Exception as e:  # noqa: BLE001
                err = e
            allh: List = [None] * self.world
            dist.all_gather_object(allh, mine, group=group)
            if err is None and any(h is None for h in allh):
                err = RuntimeError("a peer could not allocate its staging buffer")
            if err is None:
                try:
                    for r, (hb, hs) in enumerate(allh):
                        if r == self.rank:
                            self.data.append(self._buf)
                            self.sig.append(self._sig)
                        else:
                            b = C.car_open(hb)
                            self._opened.append(b)
                            sg = C.car_open(hs)
                            self._opened.append(sg)
                            self.data.append(b)
                            self.sig.append(sg)
                except Exception as e:  # noqa: BLE001
                    err = e
            oks: List = [None] * self.world
            dist.all_gather_object(oks, err is None, group=group)
        if not all(oks):
            self.close()
            raise RuntimeError(f"custom all-reduce setup failed: {err or 'on a peer rank'}")
        # pinned host-mapped word every kernel raises on a barrier timeout: ``poll()`` reads it
        # with a plain host load after each step (no device sync)
        self._flag_host, self._flag_dev = C.car_host_flag_alloc()
        self.calls = 0

    # ------------------------------------------------------------------------------------------
    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in _DTYPES and t.is_contiguous()
                and t.numel() % 8 == 0 and 0 < t.numel() * t.element_size() <= self.max_bytes)

    def plan(self, nbytes: int, numel: int):
        """(two_shot, blocks) for a message: ~2 units of 8 elements per thread (256 threads)
        up to the kernel's block limit."""
        two = nbytes > self.one_shot_max
        units = numel // 8
        blocks = max(1, min(self.max_blocks, -(-units // 512)))
        if two:
            blocks = max(1, min(blocks, units // self.world))
        return two, blocks

    def all_reduce(self, t: torch.Tensor, out: Optional[torch.Tensor] = None,
                   two_shot: Optional[bool] = None, blocks: Optional[int] = None) -> torch.Tensor:
        """Sum ``t`` over the group into ``out`` (default: in place).  Every rank must call
        with the same shape and the same (two_shot, blocks) plan."""
        if not self.eligible(t):
            raise ValueError(f"tensor not eligible for the custom all-reduce: {tuple(t.shape)} "
                             f"{t.dtype} contiguous={t.is_contiguous()}")
        out = t if out is None else out
        p_two, p_blocks = self.plan(t.numel() * t.element_size(), t.numel())
        two = p_two if two_shot is None else bool(two_shot)
        nb = p_blocks if blocks is None else int(blocks)
        self.C.car_allreduce(self.data, self.sig, self.rank, t, out, two, nb, self.timeout_s,
                             self._flag_dev)
        self.calls += 1
        return out

    def gather_eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dim() == 2 and t.dtype in _DTYPES and t.is_contiguous()
                and t.shape[1] % 8 == 0 and 0 < t.numel() * t.element_size() <= self.max_bytes)

    def all_gather_cols(self, t: torch.Tensor, out: Optional[torch.Tensor] = None,
                        blocks: Optional[int] = None) -> torch.Tensor:
        """[R, Vs] shards -> [R, W*Vs] with rank q's shard in columns q*Vs .. (q+1)*Vs."""
        if not self.gather_eligible(t):
            raise ValueError(f"tensor not eligible for the custom all-gather: {tuple(t.shape)}")
        R, Vs = t.shape
        if out is None:
            out = torch.empty(R, Vs * self.world, dtype=t.dtype, device=t.device)
        units = t.numel() // 8
        nb = blocks if blocks is not None else max(1, min(self.max_blocks, -(-units // 512)))
        self.C.car_allgather(self.data, self.sig, self.rank, t, out, int(nb), self.timeout_s,
                             self._flag_dev)
        self.calls += 1
        return out

    def poll(self) -> None:
        """Raise if a kernel launched so far and already finished hit a barrier timeout.  A plain
        read of the pinned host word: call it after each step's host sync (the serving engine
        does, right after reading the sampled tokens) so a step whose reduction went wrong never
        returns its tokens."""
        if self._flag_host and self.C.car_host_flag_read(self._flag_host):
            raise CollectiveTimeout(
                f"custom all-reduce rank {self.rank}: a barrier timed out (a peer did not "
                f"arrive within {self.timeout_s:.0f} s); this step's TP reduction is invalid")

    def check(self) -> None:
        """Raise if any barrier of this rank timed out (a peer never arrived).  Syncs."""
        err = self.C.car_err(self._sig)
        if err:
            raise RuntimeError(f"custom all-reduce rank {self.rank}: barrier timed out "
                               f"(a peer did not arrive within {self.timeout_s:.0f} s)")

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.C.car_close(p)
        for p in (self._buf, self._sig):
            if p is not None:
                self.C.car_free(p)
        self._buf = self._sig = None
        self._opened = []
        self.data, self.sig = [], []
        if getattr(self, "_flag_host", 0):
            self.C.car_host_flag_free(self._flag_host)
            self._flag_host = self._flag_dev = 0


def maybe_custom_allreduce(group, device, max_bytes: int) -> Optional[CustomAllReduce]:
    """The custom all-reduce for a TP group on GPUs, or None (CPU, world 1, disabled with
    ``LUMEN_CUSTOM_AR=0``, or peer mapping unavailable: then RCCL serves every call)."""
    if (device.type != "cuda" or group is None or dist.get_world_size(group) < 2
            or os.environ.get("LUMEN_CUSTOM_AR", "1") == "0"):
        return None
    try:
        return CustomAllReduce(group, device, max_bytes=max_bytes)
    except Exception as e:  # noqa: BLE001 - fall back to RCCL, but say so
        if dist.get_rank(group) == 0:
            print(f"[lumen] custom all-reduce unavailable ({e}); TP uses RCCL", flush=True)
        return None
