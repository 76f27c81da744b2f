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

``calibrate()`` replaces the guessed crossovers with measured ones: on the real group it times
one-shot, two-shot and RCCL at a ladder of message sizes (max over ranks), then ``pick_plan``
sets ``one_shot_max`` (one- vs two-shot) and ``rccl_from`` (the smallest size from which RCCL
won: eager calls of that size and up go to RCCL; captured decode graphs keep the custom
kernel, since RCCL is not captured).  The serving engine calibrates at TP start-up and the
bench reports the table (``extra.serve_tp.car_plan``).
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


CAL_SIZES = (8 << 10, 32 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20,
             8 << 20)


def pick_plan(table: List[dict], margin: float = 0.03) -> dict:
    """Crossovers from a calibration table (rows ``{"bytes", "one", "two"[, "rccl"]}``, times in
    us, sorted by size).  ``one_shot_max``: the largest size below the first one at which
    two-shot beats one-shot by more than ``margin`` (every size when it never does);
    ``rccl_from``: the smallest size from which RCCL beats the better custom variant by more than
    ``margin`` at that size and every larger one (None: the custom kernel wins throughout)."""
    rows = sorted(table, key=lambda r: r["bytes"])
    if not rows:
        raise ValueError("empty calibration table")
    one_max = rows[-1]["bytes"]
    for i, r in enumerate(rows):
        if r["two"] < r["one"] * (1.0 - margin):
            one_max = rows[i - 1]["bytes"] if i else 0
            break
    best = [min(r["one"] if r["bytes"] <= one_max else r["two"], r["two"]) for r in rows]
    rccl_from = None
    for i in range(len(rows) - 1, -1, -1):
        rc = rows[i].get("rccl")
        if rc is None or not rc < best[i] * (1.0 - margin):
            break
        rccl_from = rows[i]["bytes"]
    return {"one_shot_max": int(one_max), "rccl_from": rccl_from}


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
                mine = (C.car_handle(self._buf), C.car_handle(self._sig), _device_id(self.device))
            except Exception as e:  # noqa: BLE001
                err = e
            allh: List = [None] * self.world
            dist.all_gather_object(allh, mine, group=group)
            if err is None and any(h is None for h in allh):
                err = RuntimeError("a peer could not allocate its staging buffer")
            # every rank on one physical device: a shared-GPU rehearsal (processes time-share
            # the chip, so barrier timings mean nothing and calibration is skipped)
            self.shared_device = (err is None and len({h[2] for h in allh}) == 1)
            if err is None:
                try:
                    for r, (hb, hs, _) in enumerate(allh):
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
        self.rccl_from: Optional[int] = None   # eager calls of this size and up prefer RCCL
        self.calibration: Optional[dict] = None

    # ------------------------------------------------------------------------------------------
    def _time_us(self, fn, iters: int, warmup: int) -> float:
        for _ in range(warmup):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / iters

    def calibrate(self, rccl_group=None, sizes=CAL_SIZES, iters: int = 20, warmup: int = 3,
                  apply: bool = True) -> dict:
        """Time one-shot / two-shot (and RCCL on ``rccl_group``) all-reduces of bf16 messages
        of each size on this group; per size the max over ranks.  Collective over the group
        (and ``rccl_group``): every rank calls it with the same arguments.  ``apply`` installs
        ``pick_plan``'s crossovers.  Returns {"table": [...], "plan": {...}}."""
        table = []
        with torch.cuda.device(self.device):
            for nb in sizes:
                if nb > self.max_bytes or nb % 16:
                    continue
                t = torch.ones(nb // 2, dtype=torch.bfloat16, device=self.device)
                row = {"bytes": int(nb)}
                for name, two in (("one", False), ("two", True)):
                    blocks = self._blocks(t.numel(), two)
                    row[name] = self._time_us(
                        lambda: self.C.car_allreduce(self.data, self.sig, self.rank, t, t, two,
                                                     blocks, self.timeout_s, self._flag_dev),
                        iters, warmup)
                if rccl_group is not None:
                    row["rccl"] = self._time_us(lambda: dist.all_reduce(t, group=rccl_group),
                                                iters, warmup)
                table.append(row)
            # a barrier timeout on any rank is decided collectively, AFTER the max-reduction
            # every rank takes part in: raising on one rank before it would leave its peers
            # waiting in that reduction
            torch.cuda.synchronize(self.device)
            timed_out = bool(self._flag_host and self.C.car_host_flag_read(self._flag_host))
            keys = ["one", "two"] + (["rccl"] if rccl_group is not None else [])
            vals = torch.tensor([[r[k] for k in keys] + [float(timed_out)] for r in table]
                                or [[0.0] * len(keys) + [float(timed_out)]],
                                dtype=torch.float64)
            if dist.get_backend(self.group) == "nccl":
                dv = vals.to(self.device)
                dist.all_reduce(dv, op=dist.ReduceOp.MAX, group=self.group)
                vals = dv.cpu()
            else:
                dist.all_reduce(vals, op=dist.ReduceOp.MAX, group=self.group)
        if vals[:, -1].max().item() > 0:
            self.poll()  # this rank's own timeout, with its diagnostics
            raise CollectiveTimeout(f"custom all-reduce rank {self.rank}: a peer's barrier "
                                    "timed out during calibration")
        vals = vals[:, :-1]
        for r, v in zip(table, vals.tolist()):
            for k, x in zip(keys, v):
                r[k] = round(float(x), 2)
        plan = pick_plan(table)
        if apply:
            self.one_shot_max = plan["one_shot_max"]
            self.rccl_from = plan["rccl_from"]
        self.calibration = {"world": self.world, "table": table, "plan": plan}
        return self.calibration

    def prefer(self, t: torch.Tensor) -> bool:
        """Eager call: custom kernel (True) or RCCL (False) for this message, per calibration.
        Inside a graph capture the custom kernel is the only capturable choice."""
        if not self.eligible(t):
            return False
        if self.rccl_from is None or torch.cuda.is_current_stream_capturing():
            return True
        return t.numel() * t.element_size() < self.rccl_from

    # ------------------------------------------------------------------------------------------
    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in _DTYPES and t.is_contiguous()
                and t.numel() % 8 == 0 and 0 < t.numel() * t.element_size() <= self.max_bytes)

    def _blocks(self, numel: int, two: bool) -> int:
        """~2 units of 8 elements per thread (256 threads) up to the kernel's block limit; a
        two-shot block splits its span over the W ranks, so at most units / W blocks."""
        units = numel // 8
        blocks = max(1, min(self.max_blocks, -(-units // 512)))
        return max(1, min(blocks, units // self.world)) if two else blocks

    def plan(self, nbytes: int, numel: int):
        """(two_shot, blocks) for a message."""
        two = nbytes > self.one_shot_max
        return two, self._blocks(numel, two)

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

    def diagnostics(self) -> dict:
        """This rank's barrier record (synchronous device read: call after a timeout or at the
        end of a run, never per step): the first timed-out wait -- which barrier, block and
        MISSING PEER, and the low 8 bits of that block's call count -- and the longest barrier
        wait above 1 ms with the number of such waits (how far the ranks drifted apart)."""
        err, info, long_us, n_long = self.C.car_diag(self._sig)
        d = {"rank": self.rank, "timed_out": bool(err), "long_wait_ms": long_us / 1000.0,
             "long_waits": int(n_long), "calls": self.calls}
        if info >> 31:
            d.update(barrier=(info >> 24) & 0x7F, block=(info >> 16) & 0xFF,
                     missing_peer=(info >> 8) & 0xFF, epoch_lo8=info & 0xFF)
        return d

    def poll(self) -> None:
        """Raise if a kernel launched so far and already finished hit a barrier timeout.  A plain
        read of the pinned host word: call it after each step's host sync (the serving engine
        does, right after reading the sampled tokens) so a step whose reduction went wrong never
        returns its tokens."""
        if self._flag_host and self.C.car_host_flag_read(self._flag_host):
            try:
                d = self.diagnostics()
                where = (f" (barrier {d['barrier']} of block {d['block']} waited for rank "
                         f"{d['missing_peer']}; call {d['epoch_lo8']} mod 256; "
                         f"{self.calls} calls issued on this rank)") if "missing_peer" in d else ""
            except Exception:  # noqa: BLE001 - the timeout itself is the error to report
                where = ""
            raise CollectiveTimeout(
                f"custom all-reduce rank {self.rank}: a barrier timed out (a peer did not "
                f"arrive within {self.timeout_s:.0f} s){where}; this step's TP reduction is "
                "invalid")

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


def _device_id(device) -> str:
    """Identity of the PHYSICAL device (UUID where torch reports it, else PCI location)."""
    try:
        p = torch.cuda.get_device_properties(device)
        u = getattr(p, "uuid", None)
        if u is not None:
            return str(u)
        return f"{getattr(p, 'pci_domain_id', 0)}:{getattr(p, 'pci_bus_id', 0)}:" \
               f"{getattr(p, 'pci_device_id', 0)}"
    except Exception:  # noqa: BLE001
        return str(device)


def maybe_custom_allreduce(group, device, max_bytes: int) -> Optional[CustomAllReduce]:
    """The custom all-reduce for a TP group on GPUs, or None (CPU, world 1, disabled with
    ``LUMEN_CUSTOM_AR=0``, or peer mapping unavailable: then RCCL serves every call)."""
    if (device.type != "cuda" or group is None or dist.get_world_size(group) < 2
            or os.environ.get("LUMEN_CUSTOM_AR", "1") == "0"):
        return None
    try:
        car = CustomAllReduce(group, device, max_bytes=max_bytes)
    except Exception as e:  # noqa: BLE001 - fall back to RCCL, but say so
        if dist.get_rank(group) == 0:
            print(f"[lumen] custom all-reduce unavailable ({e}); TP uses RCCL", flush=True)
        return None
    # LUMEN_CAR_CALIBRATE: 1 (default) = calibrate across physical devices, fall back to RCCL
    # if it times out; always = also on a shared device (rehearsal), same fallback; force =
    # always, and a failure is fatal; 0 = never
    mode = os.environ.get("LUMEN_CAR_CALIBRATE", "1")
    if mode in ("force", "always") or (mode != "0" and not car.shared_device):
        # measured crossovers on THIS group (xGMI on a node; shared-device rehearsals measure
        # nonsense but run the same code): replaces the guessed one-shot limit
        try:
            cal = car.calibrate(rccl_group=group if dist.get_backend(group) == "nccl" else None)
        except CollectiveTimeout as e:
            # calibration is tuning only: every rank sees the same timeout after calibrate's
            # max-reduction, so all of them drop the custom kernel here together (its barrier
            # epochs are out of step anyway) and serve every reduction on RCCL.  An explicit
            # LUMEN_CAR_CALIBRATE=force keeps the failure fatal.
            if mode == "force":
                raise
            car.close()
            if dist.get_rank(group) == 0:
                import sys

                print(f"[lumen] custom all-reduce calibration failed ({e}); TP uses RCCL",
                      file=sys.stderr, flush=True)
            return None
        if dist.get_rank(group) == 0:
            import sys

            print(f"[lumen] custom all-reduce calibrated (world {car.world}): "
                  f"{cal['plan']}", file=sys.stderr, flush=True)
    return car
