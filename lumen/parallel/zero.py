"""ZeRO-1/2/3 data parallelism built directly on torch.distributed collectives (RCCL over xGMI).

Reference behaviour: DeepSpeed ZeRO stages selected by ``zero_optimization.stage`` in
configs/ds_config_zero{1,2,3}.json (trained through HF Trainer at
training/train_deepspeed_zero1.py:233, zero2.py:269, zero3.py:238):
  stage 1  optimizer state partitioned, grads reduce-scattered at the accumulation boundary
  stage 2  + gradients partitioned: bucketed reduce-scatter during every backward
  stage 3  + parameters partitioned: per-module all-gather before use, release after, prefetch,
           params below ``stage3_param_persistence_threshold`` stay resident
  offload  ``offload_optimizer`` / ``offload_param`` device=cpu (configs/ds_config_zero3.json:19-27)

MI355X-first design (not a DeepSpeed translation):
* Trainable parameters live in ONE flat f32 buffer laid out in backward-ready order and cut
  into buckets; each bucket is split evenly over ranks, so a rank's optimizer shard is the
  concatenation of its slice of every bucket.  Grads accumulate in place into a matching flat
  buffer (param.grad are views), so there are no flatten/unflatten copies.
* The fused AdamW kernel (kernels/adamw.hip) reads the global grad-norm from device memory and
  folds unscale, averaging and clipping into the update: a bf16 step has no host sync.
* ZeRO-3 partitions the frozen base weights per "unit" (embedding, each decoder layer, head):
  one flat 16-bit shard per unit per rank, ONE all_gather_into_tensor per unit (a whole
  Llama-2-7B layer = 386 MiB per collective: large enough to run RCCL over all 7 xGMI links at
  full bandwidth, unlike DeepSpeed's 5e7-element buckets), issued ahead of use (prefetch) on the
  RCCL stream while the compute stream runs the previous layer.  With ``stage3_max_live_parameters``
  >= the model (288 GB HBM makes that the normal case) the gathered units stay live from the
  forward to the backward of the same micro-step -- one gather per unit per micro-step instead of
  DeepSpeed's two -- and are re-gathered every micro-step (the shards are the only persistent
  copy).  Below that budget units are released after use and re-gathered for the backward.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops._native import native, use_native
from .dist import DistEnv

ALIGN = 64  # elements: keeps every rank slice 16-byte aligned for the 16-byte vector kernels


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# ================================================================================================
# loss scaling (fp16)
# ================================================================================================

class DynamicLossScaler:
    """DeepSpeed DynamicLossScaler semantics (configs/ds_config_zero1.json:25-32):
    scale starts at 2**initial_scale_power; an overflow skips the step and halves the scale once
    ``hysteresis`` overflows have been absorbed; ``loss_scale_window`` clean steps double it."""

    def __init__(self, init_scale=2.0 ** 16, window=1000, hysteresis=2, min_scale=1.0,
                 static_scale: float = 0.0):
        self.static = static_scale > 0
        self.scale = static_scale if self.static else float(init_scale)
        self.window, self.hysteresis, self.min_scale = window, hysteresis, min_scale
        self.cur_hysteresis = hysteresis
        self.iter = 0
        self.last_overflow_iter = -1

    def update(self, overflow: bool):
        if self.static:
            self.iter += 1
            return
        if overflow:
            if self.hysteresis == 1 or self.cur_hysteresis == 1:
                self.scale = max(self.scale / 2.0, self.min_scale)
            else:
                self.cur_hysteresis -= 1
            self.last_overflow_iter = self.iter
        else:
            if (self.iter - self.last_overflow_iter) % self.window == 0:
                self.scale *= 2.0
                self.cur_hysteresis = self.hysteresis
        self.iter += 1

    def state_dict(self):
        return dict(scale=self.scale, cur_hysteresis=self.cur_hysteresis, iter=self.iter,
                    last_overflow_iter=self.last_overflow_iter)

    def load_state_dict(self, d):
        self.scale = d["scale"]
        self.cur_hysteresis = d["cur_hysteresis"]
        self.iter = d["iter"]
        self.last_overflow_iter = d["last_overflow_iter"]


# ================================================================================================
# trainable parameters: flat buffers, buckets, shards
# ================================================================================================

@dataclass
class Bucket:
    off: int
    size: int            # padded, multiple of world * ALIGN
    params: List[nn.Parameter] = field(default_factory=list)
    shard_off: int = 0   # offset of this bucket's slice inside the rank shard
    ready: int = 0
    work: Optional[object] = None


class FlatTrainable:
    def __init__(self, params: Sequence[nn.Parameter], env: DistEnv, bucket_numel: int,
                 device: torch.device):
        self.env = env
        W = env.world_size
        self.device = device
        ps = list(params)[::-1]  # backward produces grads roughly in reverse registration order
        self.buckets: List[Bucket] = []
        cur: List[nn.Parameter] = []
        cur_n = 0
        for p in ps:
            if cur and cur_n + p.numel() > bucket_numel:
                self._close(cur, cur_n, W)
                cur, cur_n = [], 0
            cur.append(p)
            cur_n += p.numel()
        if cur:
            self._close(cur, cur_n, W)
        self.numel = sum(b.size for b in self.buckets)
        self.shard_numel = self.numel // W
        self.param = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.index: Dict[int, tuple] = {}
        so = 0
        for b in self.buckets:
            b.shard_off = so
            so += b.size // W
            o = b.off
            for p in b.params:
                n = p.numel()
                self.param[o:o + n].copy_(p.data.reshape(-1).float())
                p.data = self.param[o:o + n].view_as(p)
                p.grad = self.grad[o:o + n].view_as(p)
                self.index[id(p)] = (b, o, n)
                o += n

    def _close(self, params, n, W):
        off = self.buckets[-1].off + self.buckets[-1].size if self.buckets else 0
        self.buckets.append(Bucket(off, _round_up(max(n, 1), W * ALIGN), list(params)))

    # rank slice of a bucket inside the flat buffers
    def rank_slice(self, b: Bucket, rank: Optional[int] = None) -> slice:
        r = self.env.rank if rank is None else rank
        s = b.size // self.env.world_size
        return slice(b.off + r * s, b.off + (r + 1) * s)

    def shard_view(self, buf: torch.Tensor, b: Bucket) -> torch.Tensor:
        s = b.size // self.env.world_size
        return buf[b.shard_off:b.shard_off + s]

    def gather_shard(self, flat: torch.Tensor) -> torch.Tensor:
        """Copy this rank's slices of `flat` into a new contiguous shard tensor."""
        return torch.cat([flat[self.rank_slice(b)] for b in self.buckets])


# ================================================================================================
# ZeRO-3 parameter coordinator (frozen/base weights)
# ================================================================================================

class _LocalGather:
    """World-1 stand-in for an async ``all_gather_into_tensor`` (the shard IS the whole unit):
    a copy on a side stream ordered after the issuing stream, with ``wait()`` making the
    current stream wait on it -- the same stream semantics ProcessGroupNCCL gives, so the
    coordinator's schedule can be exercised on one GPU (``LUMEN_ZERO3_SINGLE=1``)."""

    _stream = None

    def __init__(self, out: torch.Tensor, shard: torch.Tensor):
        if out.is_cuda:
            if _LocalGather._stream is None:
                _LocalGather._stream = torch.cuda.Stream(device=out.device)
            s = _LocalGather._stream
            s.wait_stream(torch.cuda.current_stream(out.device))
            with torch.cuda.stream(s):
                out.copy_(shard, non_blocking=True)
                self.ev = torch.cuda.Event()
                self.ev.record(s)
            shard.record_stream(s)
            out.record_stream(s)
        else:
            out.copy_(shard)
            self.ev = None

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)


class _Unit:
    def __init__(self, idx):
        self.idx = idx
        self.params: List[nn.Parameter] = []
        self.deps: List[int] = []
        self.numel = 0
        self.padded = 0
        self.shard: Optional[torch.Tensor] = None      # [padded / W] (device, or pinned host)
        self.bufs: List[Optional[torch.Tensor]] = []   # per slot: [padded] gathered (device)
        self.works: List[Optional[object]] = []
        self.states: List[str] = []                    # per slot: empty | inflight | ready
        self.bound = -1                                # slot the params currently view, or -1
        self.dtype = None
        # W^T copies made off the critical path (keep / pipelined): (param idx, off, wt_off)
        self.tn: List[tuple] = []
        self.wt_numel = 0
        self.wt_bufs: List[Optional[torch.Tensor]] = []
        self.wt_events: List[Optional[object]] = []


class ParamCoordinator:
    """Gathers / releases ZeRO-3 partitioned units around the model's unit loop.

    The model calls ``pre_forward(i)`` / ``post_forward(i, out)``; gradient hooks on unit outputs
    call ``pre_backward(i)`` (before unit i's backward runs); the engine calls
    ``end_micro_step()`` after ``loss.backward()``.  Every gather is one
    ``all_gather_into_tensor`` of a unit's shards on the process group's RCCL stream; the compute
    stream waits on it only right before the unit runs.  The shards are the only persistent copy
    of the frozen weights: every micro-step re-materialises every unit over xGMI.

    Schedules (chosen from ``stage3_max_live_parameters``, DeepSpeed's live-parameter budget):

    * ``release`` (budget < model): gather before use, prefetch the next ``depth`` units, free
      after the forward, gather again for the backward (DeepSpeed's schedule).
    * ``keep`` (model <= budget < 2x model): one buffer per unit, gathered once per micro-step
      and kept from the forward through the backward.  As soon as unit i's backward has run,
      its buffer is re-gathered for the next micro-step (the frozen values cannot change in
      between), so the next step's gathers overlap this step's backward.
    * ``pipelined`` (budget >= 2x model, the 7B-on-288 GB case): two buffers per unit; the
      whole next micro-step's gathers are issued, in forward order, when the current one
      starts, so one step of compute hides one step of xGMI traffic.  This is what makes
      2-4 GPU ZeRO-3 compute-bound: a 2-GPU all-gather of 6.3 GB crosses ONE xGMI link.
    """

    def __init__(self, model: nn.Module, env: DistEnv, persistence_threshold: int,
                 max_live: int, prefetch_numel: int, offload_param: bool = False,
                 pin_memory: bool = True, schedule: Optional[str] = None):
        self.env = env
        self.model = model
        self.offload = offload_param
        W = env.world_size
        self.local = not (dist.is_available() and dist.is_initialized()) and W == 1
        mark_zero_shapes(model)
        units_mods = model.zero_units()
        owner: Dict[int, int] = {}
        self.units: List[_Unit] = []
        self.persistent: List[nn.Parameter] = []
        for i, mods in enumerate(units_mods):
            u = _Unit(i)
            for m in mods:
                for p in m.parameters():
                    if p.requires_grad:
                        continue  # trainable params are handled by FlatTrainable (persistent)
                    if p.numel() < persistence_threshold:
                        if id(p) not in owner:
                            owner[id(p)] = -1
                            self.persistent.append(p)
                        continue
                    if id(p) in owner:
                        if owner[id(p)] >= 0 and owner[id(p)] != i and owner[id(p)] not in u.deps:
                            u.deps.append(owner[id(p)])
                        continue
                    owner[id(p)] = i
                    u.params.append(p)
            self.units.append(u)
        total = 0
        for u in self.units:
            if not u.params:
                continue
            u.dtype = u.params[0].dtype
            assert all(p.dtype == u.dtype for p in u.params), "a unit must have one dtype"
            u.numel = sum(p.numel() for p in u.params)
            u.padded = _round_up(u.numel, W * ALIGN)
            total += u.padded
            s = u.padded // W
            r0 = env.rank * s
            flat = torch.cat([p.data.reshape(-1) for p in u.params])
            if flat.numel() < u.padded:
                flat = torch.cat([flat, flat.new_zeros(u.padded - flat.numel())])
            shard = flat[r0:r0 + s].clone()
            if offload_param:
                shard = shard.cpu()
                if pin_memory and torch.cuda.is_available():
                    shard = shard.pin_memory()
            u.shard = shard
            del flat
            for p in u.params:
                p.data = torch.empty(0, dtype=u.dtype, device=p.device)
                p._lumen_gathered = True  # storage swapped per gather: no derived caches
        self.total_numel = total
        self.max_live = max_live if max_live >= 0 else self._hbm_live_budget(units_dtype_bytes(
            self.units))
        if schedule is None:
            schedule = ("pipelined" if 2 * total <= self.max_live else
                        "keep" if total <= self.max_live else "release")
        assert schedule in ("release", "keep", "pipelined"), schedule
        self.schedule = schedule
        self.keep = schedule != "release"
        n_slots = 2 if schedule == "pipelined" else 1
        for u in self.units:
            u.bufs = [None] * n_slots
            u.works = [None] * n_slots
            u.states = ["empty"] * n_slots
            u.wt_bufs = [None] * n_slots
            u.wt_events = [None] * n_slots
        self._tstream = None
        self.transposed_numel = 0
        self.slot = 0
        # prefetch depth (release mode): upcoming units whose gathered size fits the bucket
        sizes = [u.padded for u in self.units if u.padded]
        avg = (sum(sizes) / len(sizes)) if sizes else 1
        self.depth = max(1, int(prefetch_numel // max(avg, 1)))
        if self.keep:
            self.depth = max(self.depth, 2)
        self.last = len(self.units) - 1
        self.device = env.device
        self._bwd_seen = set()
        self._in_step = False
        self.gathered_bytes = 0    # bytes materialised by gathers (all ranks' shards)
        self.gathers = 0
        from ..utils.debug import zero3_poison_enabled

        self.poison = zero3_poison_enabled()

    def _hbm_live_budget(self, elem_bytes: int) -> int:
        """``stage3_max_live_parameters: "auto"``: elements of gathered weights that fit in the
        free HBM left after the shards, minus an activation reserve (max(48 GiB, 25% of the
        device)).  On MI355X (288 GB) that is both buffers of the pipelined schedule for
        Llama-2-7B and one full copy (keep) for Llama-2-70B.  Unlimited off-GPU."""
        if self.env.device.type != "cuda":
            return 1 << 62
        free, total = torch.cuda.mem_get_info(self.env.device)
        # blocks the caching allocator holds but no tensor uses (the full weights just sharded)
        free += torch.cuda.memory_reserved(self.env.device) - torch.cuda.memory_allocated(
            self.env.device)
        reserve = float(os.environ.get("LUMEN_ZERO3_RESERVE_GB", "0")) * 2**30 or max(
            48 * 2**30, 0.25 * total)
        return max(0, int((free - reserve) // max(elem_bytes, 1)))

    # ---- gather / bind / release ------------------------------------------------------------
    def _issue(self, i: int, slot: Optional[int] = None):
        if i < 0 or i > self.last:
            return
        slot = self.slot if slot is None else slot
        u = self.units[i]
        for d in u.deps:
            self._issue(d, slot)
        if not u.params or u.states[slot] != "empty":
            return
        if u.bufs[slot] is None:
            u.bufs[slot] = torch.empty(u.padded, dtype=u.dtype, device=self.device)
        if self.poison:  # race detector: stale reads of this buffer now see NaN
            u.bufs[slot].fill_(float("nan"))
        shard = u.shard
        if self.offload:
            shard = shard.to(self.device, non_blocking=True)
        if self.local:
            u.works[slot] = _LocalGather(u.bufs[slot], shard)
        else:
            u.works[slot] = dist.all_gather_into_tensor(u.bufs[slot], shard, async_op=True)
        self.gathered_bytes += u.padded * u.bufs[slot].element_size()
        self.gathers += 1
        u.states[slot] = "inflight"
        if u.tn:
            self._transpose_after_gather(u, slot)

    def _transpose_after_gather(self, u: _Unit, slot: int):
        """On a side stream: wait for the gather, write W^T of the unit's projections (for the
        backward's TN input-gradient GEMMs).  Overlaps compute instead of sitting in the
        backward; the compute stream waits on the event only when it binds the unit."""
        from ..ops.transpose import transpose_2d

        cur = torch.cuda.current_stream(self.device)
        if self._tstream is None:
            self._tstream = torch.cuda.Stream(device=self.device)
        side = self._tstream
        if u.wt_bufs[slot] is None:
            u.wt_bufs[slot] = torch.empty(u.wt_numel, dtype=u.dtype, device=self.device)
        side.wait_stream(cur)      # earlier readers of this slot's W^T are done
        with torch.cuda.stream(side):
            u.works[slot].wait()   # side stream waits on the collective
            full, wt = u.bufs[slot], u.wt_bufs[slot]
            for k, off, wt_off in u.tn:
                rows, cols = u.params[k]._zero_shape
                transpose_2d(full[off:off + rows * cols].view(rows, cols),
                             out=wt[wt_off:wt_off + rows * cols].view(cols, rows))
            ev = torch.cuda.Event()
            ev.record(side)
        u.wt_events[slot] = ev

    def enable_transposes(self, params: Sequence[nn.Parameter]) -> int:
        """Keep W^T of these gathered weights next to the gathered buffer (keep / pipelined
        schedules, when HBM allows: one more copy of the projections per slot).  Returns the
        number of weights covered."""
        if self.schedule == "release" or self.device.type != "cuda":
            return 0
        want = {id(p) for p in params}
        need = 0
        plan = []
        for u in self.units:
            tn, o, wo = [], 0, 0
            for k, p in enumerate(u.params):
                shape = p._zero_shape
                n = math.prod(shape)
                if (id(p) in want and len(shape) == 2 and shape[0] % 8 == 0
                        and shape[1] % 8 == 0 and p.dtype in (torch.bfloat16, torch.float16)):
                    tn.append((k, o, wo))
                    wo += n
                o += n
            plan.append((u, tn, wo))
            need += wo * (u.dtype.itemsize if u.dtype is not None else 2) * len(u.bufs)
        free, total = torch.cuda.mem_get_info(self.device)
        # the gathered buffers themselves are not allocated yet: keep room for them and for
        # activations (max(48 GiB, 25% of HBM))
        gathered = sum(u.padded * u.dtype.itemsize for u in self.units if u.params) * len(
            self.units[0].bufs)
        if need + gathered > free - max(48 * 2**30, 0.25 * total):
            return 0
        n = 0
        for u, tn, wo in plan:
            u.tn, u.wt_numel = tn, wo
            n += len(tn)
            self.transposed_numel += wo
        return n

    def _wait(self, i: int):
        """Make unit i's params view the current slot's gathered buffer."""
        u = self.units[i]
        for d in u.deps:
            self._wait(d)
        if not u.params:
            return
        s = self.slot
        if u.states[s] == "empty":
            self._issue(i, s)
        if u.states[s] == "inflight":
            u.works[s].wait()
            u.works[s] = None
            u.states[s] = "ready"
        if u.bound != s:
            o = 0
            full = u.bufs[s]
            for p in u.params:
                shape = p._zero_shape
                n = math.prod(shape)
                p.data = full[o:o + n].view(shape)
                o += n
            if u.tn:
                if u.wt_events[s] is not None:
                    torch.cuda.current_stream(self.device).wait_event(u.wt_events[s])
                    u.wt_events[s] = None
                wt = u.wt_bufs[s]
                for k, off, wt_off in u.tn:
                    rows, cols = u.params[k]._zero_shape
                    u.params[k]._lumen_wt = wt[wt_off:wt_off + rows * cols].view(cols, rows)
            u.bound = s

    def _unbind(self, u: _Unit):
        if u.bound >= 0:
            for p in u.params:
                p.data = torch.empty(0, dtype=u.dtype, device=p.device)
                p._lumen_wt = None
            u.bound = -1

    def _release(self, i: int):
        """Drop unit i's current-slot contents (release schedule: free the memory too)."""
        if i < 0 or i > self.last:
            return
        u = self.units[i]
        if not u.params:
            return
        s = self.slot
        if u.states[s] == "inflight":
            u.works[s].wait()
            u.works[s] = None
        self._unbind(u)
        if self.schedule == "release":
            u.bufs[s] = None  # return memory to the caching allocator (stream-ordered)
        u.states[s] = "empty"

    def _refresh(self, i: int):
        """keep schedule: unit i is done for this micro-step -> re-gather it for the next one
        into the same buffer (issued after the compute that read it, on the RCCL stream)."""
        if i < 1 or i > self.last:
            return
        u = self.units[i]
        if not u.params or u.states[self.slot] != "ready":
            return
        self._release(i)
        self._issue(i)

    # ---- model hooks ------------------------------------------------------------------------
    def begin_micro_step(self):
        self._bwd_seen.clear()
        self._in_step = True
        if self.schedule == "pipelined":
            for i in range(self.last + 1):
                self._issue(i, self.slot)
            for i in range(self.last + 1):
                self._issue(i, 1 - self.slot)  # next micro-step, behind this one's
        else:
            for i in range(min(self.depth, self.last + 1)):
                self._issue(i)

    def pre_forward(self, i: int):
        if i == 0 and not self._in_step:
            self.begin_micro_step()
        self._wait(i)
        if self.schedule != "pipelined":
            for j in range(i + 1, min(i + 1 + self.depth, self.last + 1)):
                self._issue(j)

    def post_forward(self, i: int, out):
        if self.schedule == "release" and i != self.last:
            self._release(i)
        if torch.is_grad_enabled():
            tensors = out if isinstance(out, (tuple, list)) else (out,)
            for t in tensors:
                if isinstance(t, torch.Tensor) and t.requires_grad:
                    t.register_hook(self._make_bwd_hook(i))
        elif i == self.last:
            self.end_micro_step()
        return out

    def _make_bwd_hook(self, i):
        def hook(grad):
            self.pre_backward(i)
            return grad
        return hook

    def pre_backward(self, i: int):
        """Runs when the gradient of unit i's output is complete, i.e. after unit i+1's backward
        and before unit i's."""
        if i in self._bwd_seen:
            return
        if not self._bwd_seen:
            # first hook of this backward: close the micro-step when the whole pass is done
            # (unit 1's backward runs after the last hook fires)
            torch.autograd.Variable._execution_engine.queue_callback(self.end_micro_step)
        self._bwd_seen.add(i)
        if self.schedule == "release":
            self._release(i + 1)
        elif self.schedule == "keep":
            self._refresh(i + 1)
        self._wait(i)
        if self.schedule == "release":
            for j in range(i - 1, max(i - 1 - self.depth, -1), -1):
                if j >= 1:  # unit 0 (embedding) has no backward
                    self._issue(j)

    def end_micro_step(self):
        """After the backward (or a no-grad forward): nothing of this micro-step is read any
        more.  Idempotent (the autograd callback and the engine both call it)."""
        if not self._in_step:
            return
        self._in_step = False
        if self.schedule == "keep":
            for i in range(self.last + 1):  # units without a backward, then unit 1
                u = self.units[i]
                if u.params and u.states[self.slot] == "ready":
                    self._release(i)
                    self._issue(i)
        elif self.schedule == "pipelined":
            for u in self.units:
                self._unbind(u)
                u.states[self.slot] = "empty"   # re-gathered (for micro-step t+2) at t+1's start
            self.slot = 1 - self.slot
        else:
            for i in range(self.last + 1):
                self._release(i)

    def gather_all_full(self) -> None:
        """Materialise every unit (checkpoint save with gather_16bit_weights_on_model_save)."""
        for i in range(self.last + 1):
            self._issue(i)
            self._wait(i)

    def release_all(self):
        for i in range(self.last + 1):
            self._release(i)
        self._in_step = False

    def drain(self):
        """Complete every in-flight gather (all slots): before process-group teardown."""
        for u in self.units:
            for s, w in enumerate(u.works):
                if w is not None:
                    w.wait()
                    u.works[s] = None
                    u.states[s] = "ready"


def units_dtype_bytes(units: Sequence[_Unit]) -> int:
    return max((u.dtype.itemsize for u in units if u.params), default=2)


def mark_zero_shapes(model: nn.Module):
    for p in model.parameters():
        p._zero_shape = tuple(p.shape)


# ================================================================================================
# optimizer state on a shard
# ================================================================================================

class ShardAdamW:
    """AdamW over this rank's f32 shard: HIP fused kernel on GPU, C++ AVX-512 kernel when
    offloaded to CPU, torch math on CPU tensors (tests)."""

    def __init__(self, numel: int, device: torch.device, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, offload: bool = False, pin_memory: bool = True):
        self.b1, self.b2 = betas
        self.eps, self.wd = eps, weight_decay
        self.offload = offload
        sdev = torch.device("cpu") if offload else device
        mk = lambda: torch.zeros(numel, dtype=torch.float32, device=sdev)  # noqa: E731
        self.master = mk()
        self.m, self.v = mk(), mk()
        if offload and pin_memory and torch.cuda.is_available():
            self.master, self.m, self.v = (t.pin_memory() for t in (self.master, self.m, self.v))
        self.step_count = 0

    def step(self, grad: torch.Tensor, lr: float, inv_scale: float,
             norm_sq: Optional[torch.Tensor], max_norm: float) -> None:
        self.step_count += 1
        t = self.step_count
        bc1, bc2 = 1 - self.b1 ** t, 1 - self.b2 ** t
        p = self.master
        if self.offload:
            g = grad.to("cpu", non_blocking=False) if grad.is_cuda else grad
            coef = inv_scale
            if norm_sq is not None:
                nsq = float(norm_sq.item())
                if not math.isfinite(nsq):
                    self.step_count -= 1
                    return
                gn = math.sqrt(nsq) * inv_scale
                if max_norm > 0 and gn > max_norm:
                    coef *= max_norm / (gn + 1e-6)
            C = native()
            if C is not None:
                C.cpu_adamw(p, g.contiguous(), self.m, self.v, lr, self.b1, self.b2, self.eps,
                            self.wd, bc1, bc2, coef)
            else:
                _adamw_torch(p, g, self.m, self.v, lr, self.b1, self.b2, self.eps, self.wd, bc1,
                             bc2, coef)
            return
        if use_native(p):
            native().adamw(p, grad, self.m, self.v, None, lr, self.b1, self.b2, self.eps, self.wd,
                           bc1, bc2, inv_scale, norm_sq, max_norm)
            return
        coef = inv_scale
        if norm_sq is not None:
            nsq = float(norm_sq.item())
            if not math.isfinite(nsq):
                self.step_count -= 1
                return
            gn = math.sqrt(nsq) * inv_scale
            if max_norm > 0 and gn > max_norm:
                coef *= max_norm / (gn + 1e-6)
        _adamw_torch(p, grad, self.m, self.v, lr, self.b1, self.b2, self.eps, self.wd, bc1, bc2, coef)

    def state_dict(self):
        return dict(master=self.master.cpu(), exp_avg=self.m.cpu(), exp_avg_sq=self.v.cpu(),
                    step=self.step_count, betas=(self.b1, self.b2), eps=self.eps, wd=self.wd)

    def load_state_dict(self, d):
        self.master.copy_(d["master"])
        self.m.copy_(d["exp_avg"])
        self.v.copy_(d["exp_avg_sq"])
        self.step_count = int(d["step"])


def _adamw_torch(p, g, m, v, lr, b1, b2, eps, wd, bc1, bc2, coef):
    g = g.float() * coef
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    p.mul_(1 - lr * wd)
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


def grad_norm_sq(t: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    if use_native(t):
        native().grad_norm_sq(t, out)
    else:
        out.add_(t.float().pow(2).sum())
    return out
