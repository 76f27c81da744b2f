"""ZeRO-3 parameter coordinator: partitioned frozen weights, gathered around each model unit.

Reference behaviour: DeepSpeed stage 3 as configured by configs/ds_config_zero3.json:16-37
(``stage3_max_live_parameters``, ``stage3_max_reuse_distance``, ``stage3_prefetch_bucket_size``,
``stage3_param_persistence_threshold``, ``offload_param``) and exercised by the notebook's
ZeRO-3 matrix (training/train.ipynb:900-960).

MI355X-first design (not a DeepSpeed translation):

* One flat 16-bit shard per unit (embedding, each decoder layer, final norm + head) per rank and
  ONE ``all_gather_into_tensor`` per unit.  A Llama-2-7B layer is 386 MiB per collective: large
  enough for RCCL to drive all 7 xGMI links of an MI355X at full rate (DeepSpeed's 5e7-element
  buckets are latency-bound there).
* Weight gathers run on their OWN process group (a separate RCCL communicator, hence a separate
  RCCL stream).  Gradient reduce-scatters, the grad-norm all-reduce and the adapter publish
  all-gather stay on the default group, so a backward's reduce-scatter never queues behind the
  next micro-step's 6-12 GB of weight traffic.
* Schedules, picked from the live-parameter budget (``stage3_max_live_parameters``; ``"auto"``
  sizes it from free HBM):

  ``keep`` (budget >= model: Llama-2-7B on 288 GB at any world size, Llama-2-70B from 8
      GPUs).  One buffer per unit, gathered on first use (prefetched ``depth`` units ahead)
      and then RESIDENT: the partitioned weights are the frozen base model -- LoRA never writes
      them -- so a gathered buffer can never go stale, and re-gathering it every micro-step (as
      DeepSpeed does, to free the memory) would move 13.5 GB per step over xGMI to rebuild
      bytes already in HBM.  The adapter tail of the K-extended (folded) weights is rewritten
      in place whenever ``lora_B`` changes.  W^T of the projections, when enabled, is also
      written once.  Steady-state traffic: the LoRA gradient reduce-scatter and the adapter
      publish only.  (Until round 3 this schedule re-gathered after every unit's backward, and
      a ``pipelined`` variant double-buffered every unit: 102-103 ms/step forced at world 1
      against 91-93 ms for no gathers, profiles/r3_zero3.)
  ``hybrid`` (budget < model but > a two-buffer ring plus one decoder unit: Llama-2-70B on 2-4
      GPUs, or a user-set live budget, e.g. the reference's 1e9).  As many decoder units as the
      budget holds beyond the ring are resident (gathered once, W^T once, like ``keep``); they
      are spread evenly so each remaining unit's per-use all-gather overlaps the compute of the
      resident units before it, and the look-ahead counts ring units only.  The cost scales
      with the bytes that do not fit instead of jumping from ``keep`` to ``release``.
  ``release`` (budget below even that).  A preallocated ring of ``P = budget / unit`` gather
      buffers (no allocator churn); prefetch depth from ``stage3_prefetch_bucket_size``; the
      last units of the forward stay live across the forward->backward turn when they fall
      within ``stage3_max_reuse_distance`` (DeepSpeed's reuse semantics), everything else is
      gathered twice per micro-step.  ``hybrid`` runs the same ring for its non-resident units.
  ``identity`` (world size 1).  The one-rank partition IS the unit: parameters view the shard
      permanently and no gather runs.  ``LUMEN_ZERO3_SINGLE=1`` instead forces real per-step
      materialisation (a side-stream copy with RCCL's stream semantics) so the schedules
      above run on a one-GPU box.

* ``offload_param``: pinned host shards are copied H2D on a dedicated copy stream into a ring of
  device staging buffers and the all-gather is issued from that stream, so neither the copy nor
  the collective waits on -- or stalls -- the compute stream.
* Observability: bytes gathered / received per step and the EXPOSED wait (GPU time the compute
  stream spent blocked on a gather, from timing events around ``work.wait()``) when
  ``track_waits`` is on (bench.py reports both).
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import DistEnv

ALIGN = 64  # elements: every rank slice stays 16-byte aligned


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class _LocalGather:
    """World-1 stand-in for an async ``all_gather_into_tensor`` (the shard IS the whole unit):
    a copy on a side stream ordered after the issuing stream; ``wait()`` makes the current stream
    wait on it -- the stream semantics ProcessGroupNCCL gives."""

    _streams: Dict[str, torch.cuda.Stream] = {}

    def __init__(self, out: torch.Tensor, shard: torch.Tensor):
        if out.is_cuda:
            key = str(out.device)
            s = _LocalGather._streams.get(key)
            if s is None:
                s = _LocalGather._streams[key] = torch.cuda.Stream(device=out.device)
            s.wait_stream(torch.cuda.current_stream(out.device))
            with torch.cuda.stream(s):
                out[:shard.numel()].copy_(shard, non_blocking=True)
                self.ev = torch.cuda.Event()
                self.ev.record(s)
        else:
            out[:shard.numel()].copy_(shard)
            self.ev = None

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)


class _EventWork:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class _Unit:
    def __init__(self, idx):
        self.idx = idx
        self.params: List[nn.Parameter] = []
        self.deps: List[int] = []
        self.numel = 0
        self.padded = 0
        self.shard: Optional[torch.Tensor] = None      # [padded / W] (device, or pinned host)
        self.buf: Optional[torch.Tensor] = None        # [>= padded] gathered (device)
        self.work: Optional[object] = None
        self.state = "empty"                           # empty | inflight | ready
        self.bound = False                             # params view ``buf``
        self.dtype = None
        # W^T copies made off the critical path (keep): (param idx, off, wt_off)
        self.tn: List[tuple] = []
        # LoRA-folded linears of this unit: their weights are stored as [N, K + KP] rows (the
        # adapter tail of the K-extended GEMM); a bind marks the tail for a refill
        self.folds: List[nn.Module] = []
        self.wt_numel = 0
        self.wt_buf: Optional[torch.Tensor] = None
        self.wt_event: Optional[object] = None
        # gathered once and kept (keep: every unit; hybrid: the units the live budget holds
        # beyond the ring); never released, W^T written once
        self.resident = False
        # ring units: a second shard holding the unit's projections TRANSPOSED ([K, N] each):
        # the backward gathers that instead of W, so its input-gradient GEMMs run in the TN form
        # straight from the gathered buffer (no per-step transpose, no NN GEMMs)
        self.shard_t: Optional[torch.Tensor] = None
        self.padded_t = 0
        self.layout = "w"                              # contents of buf: "w" | "wt"


class ParamCoordinator:
    """Gathers / releases ZeRO-3 partitioned units around the model's unit loop.

    The model calls ``pre_forward(i)`` / ``post_forward(i, out)``; gradient hooks on unit outputs
    call ``pre_backward(i)`` (before unit i's backward runs); the engine calls
    ``end_micro_step()`` after ``loss.backward()``.  See the module docstring for schedules."""

    SCHEDULES = ("release", "hybrid", "keep", "identity")

    def __init__(self, model: nn.Module, env: DistEnv, persistence_threshold: int,
                 max_live: int, prefetch_numel: int, offload_param: bool = False,
                 pin_memory: bool = True, schedule: Optional[str] = None,
                 group=None, max_reuse_distance: int = int(1e9), force_partition: bool = False):
        self.env = env
        self.model = model
        self.offload = offload_param
        W = env.world_size
        self.world = W
        self.group = group
        self.dist = dist.is_available() and dist.is_initialized() and W > 1
        self.local = not self.dist
        if W == 1 and not (force_partition or offload_param):
            schedule = "identity"
        elif schedule == "identity":
            raise ValueError("the identity schedule needs world size 1 and no param offload")
        mark_zero_shapes(model)
        fold_lin = _mark_fold_weights(model)
        owner: Dict[int, int] = {}
        self.units: List[_Unit] = []
        self.persistent: List[nn.Parameter] = []
        for i, mods in enumerate(model.zero_units()):
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
                    if id(p) in fold_lin:
                        u.folds.append(fold_lin[id(p)])
            self.units.append(u)
        total = 0
        # transposed backward shards: only where a ring schedule is already certain here (forced
        # release / hybrid, or an explicit live budget below the model) -- an "auto" budget is
        # sized from the HBM left after sharding, and building W^T shards first would shrink it
        est_total = sum(_round_up(sum(_store_numel(p) for p in u.params), W * ALIGN)
                        for u in self.units if u.params)
        want_t = (os.environ.get("LUMEN_ZERO3_BWD_WT", "1") != "0" and not offload_param
                  and env.device.type == "cuda" and schedule not in ("identity", "keep")
                  and (schedule in ("release", "hybrid") or 0 <= max_live < est_total))
        for u in self.units:
            if not u.params:
                continue
            u.dtype = u.params[0].dtype
            assert all(p.dtype == u.dtype for p in u.params), "a unit must have one dtype"
            u.numel = sum(_store_numel(p) for p in u.params)
            u.padded = _round_up(u.numel, W * ALIGN)
            total += u.padded
            s = u.padded // W
            r0 = env.rank * s
            flat = torch.cat([_stored(p.data, getattr(p, "_lumen_fold_kp", 0)).reshape(-1)
                              for p in u.params])
            if flat.numel() < u.padded:
                flat = torch.cat([flat, flat.new_zeros(u.padded - flat.numel())])
            shard = flat[r0:r0 + s].clone() if W > 1 else flat
            if offload_param:
                shard = shard.cpu()
                if pin_memory and torch.cuda.is_available():
                    shard = shard.pin_memory()
            u.shard = shard
            del flat
            if want_t and 0 < u.idx < len(self.units) - 1 and _t_eligible(u):
                ft = torch.cat([p.data.t().contiguous().reshape(-1) for p in u.params])
                u.padded_t = _round_up(ft.numel(), W * ALIGN)
                if ft.numel() < u.padded_t:
                    ft = torch.cat([ft, ft.new_zeros(u.padded_t - ft.numel())])
                st_ = u.padded_t // W
                u.shard_t = ft[env.rank * st_:(env.rank + 1) * st_].clone() if W > 1 else ft
                del ft
            if schedule == "identity":
                self._bind_views(u, shard)       # the one-rank partition is the unit
            else:
                for p in u.params:
                    p.data = torch.empty(0, dtype=u.dtype, device=p.device)
                    p._lumen_gathered = True     # storage swapped per gather: no derived caches
        self.total_numel = total
        self.elem_bytes = units_dtype_bytes(self.units)
        self.max_live = max_live if max_live >= 0 else self._hbm_live_budget(self.elem_bytes)
        self.schedule_reason = ("world size 1: the one-rank partition is the whole unit"
                                if schedule == "identity" else
                                "forced (LUMEN_ZERO3_SCHEDULE or caller)")
        unit_sizes = [u.padded for u in self.units]
        if schedule is None:
            schedule, self.schedule_reason = self.auto_schedule(total, self.max_live, W,
                                                                unit_sizes)
        assert schedule in self.SCHEDULES, schedule
        self.schedule = schedule
        self.identity = schedule == "identity"
        self.keep = schedule == "keep"
        self.ring = schedule in ("release", "hybrid")   # some units re-gathered every use
        self._tstream = None
        self._cstream = None
        self.transposed_numel = 0
        self.last = len(self.units) - 1
        self.device = env.device
        sizes = [u.padded for u in self.units if u.padded]
        self.max_unit = max(sizes) if sizes else 0
        avg = (sum(sizes) / len(sizes)) if sizes else 1
        # prefetch depth: upcoming units whose gathered size fits the prefetch bucket
        self.depth = max(1, int(prefetch_numel // max(avg, 1)))
        # release / hybrid: ring of P gather buffers sized from the live budget (hybrid: what
        # the resident units leave of it); units kept across the forward->backward turn (those
        # within the reuse distance that the ring can hold)
        self.pool_size = 0
        self.turn_keep = 0
        self._pool: Dict[torch.dtype, List[torch.Tensor]] = {}
        self._pool_alloc = 0
        self.pool_overflows = 0
        if self.keep:
            for u in self.units:
                u.resident = bool(u.params)
        elif schedule == "hybrid":
            for i in self.resident_plan(unit_sizes, self.max_live):
                self.units[i].resident = True
        self.resident_numel = sum(u.padded for u in self.units if u.resident)
        for u in self.units:
            if u.resident or not self.ring:
                u.shard_t, u.padded_t = None, 0
        self._in_bwd = False
        if self.ring:
            ring_sizes = [u.padded for u in self.units if u.padded and not u.resident]
            n_units = len(ring_sizes)
            ring_avg = (sum(ring_sizes) / n_units) if n_units else 1
            P = int((self.max_live - self.resident_numel) // max(self.max_unit, 1))
            P = max(2, min(P, max(n_units, 2)))
            self.pool_size = P
            # DeepSpeed reuse distance: elements accessed between two uses of a unit.  Unit
            # last-k is reused after ~2k units (k more forward, k backward).  Reuse saves xGMI
            # bytes, prefetch depth only hides latency: the ring serves reuse first, then depth
            reuse_units = int(max_reuse_distance // max(2 * avg, 1))
            self.turn_keep = max(0, min(P - 2, reuse_units))
            self.depth = max(1, min(int(prefetch_numel // max(ring_avg, 1)),
                                    P - 1 - self.turn_keep))
        elif self.keep:
            self.depth = max(self.depth, 2)
        # staging ring for offloaded shards (device side of the H2D copy)
        self._staging: List[Optional[torch.Tensor]] = []
        self._staging_work: List[Optional[object]] = []
        self._staging_i = 0
        self._bwd_seen = set()
        self._in_step = False
        self.gathered_bytes = 0    # bytes materialised by gathers (all ranks' shards)
        self.gathers = 0
        self.gathers_t = 0         # ... of them transposed backward gathers
        self.track_waits = False
        self._wait_events: List[tuple] = []
        self._wait_host_s = 0.0
        from ..utils.debug import zero3_poison_enabled

        self.poison = zero3_poison_enabled() and not self.identity

    # ---- sizing -----------------------------------------------------------------------------
    @staticmethod
    def auto_schedule(total: int, max_live: int, world: int,
                      unit_sizes: Optional[Sequence[int]] = None):
        """(schedule, reason) from the live-parameter budget and the world size.

        * budget >= model: ``keep``: one gathered copy of the frozen weights, gathered once and
          kept resident (the world size only sets how fast that first gather is).
        * budget < model, but above a two-buffer ring plus at least one decoder unit:
          ``hybrid``: as many units resident as the budget holds beyond the ring, the rest
          re-gathered at every use -- the cost moves smoothly from ``keep`` to ``release``
          instead of falling off a cliff one element below the model size.
        * otherwise ``release`` (every unit gathered again at each use)."""
        if total <= max_live:
            return "keep", (f"model {total:.3g} elements <= live budget {max_live:.3g}: frozen "
                            f"weights gathered once (world {world}) and kept resident")
        why = f"model {total:.3g} elements > live budget {max_live:.3g}"
        if unit_sizes is not None:
            res = ParamCoordinator.resident_plan(unit_sizes, max_live)
            if res:
                n = sum(1 for s in unit_sizes if s)
                return "hybrid", (f"{why}: {len(res)} of {n} units resident, the rest through "
                                  "a ring of gather buffers")
        return "release", why

    @staticmethod
    def resident_plan(unit_sizes: Sequence[int], max_live: int) -> List[int]:
        """Units kept resident under ``hybrid``: decoder units (1 .. last-1 -- each saves a
        forward AND a backward gather per micro-step; the embedding has no backward and the head
        is consumed at the turn anyway), as many as the budget holds after a two-buffer ring,
        spread evenly so each re-gathered unit's all-gather overlaps resident units' compute."""
        sizes = list(unit_sizes)
        mx = max(sizes, default=0)
        cand = [i for i in range(1, len(sizes) - 1) if sizes[i]]
        if not cand or mx == 0:
            return []
        avail = max_live - 2 * mx
        per = max(sizes[i] for i in cand)
        n = int(min(len(cand), max(avail, 0) // per))
        if n <= 0:
            return []
        m = len(cand)
        return [cand[min(m - 1, int((k + 0.5) * m / n))] for k in range(n)]

    def _hbm_live_budget(self, elem_bytes: int) -> int:
        """``stage3_max_live_parameters: "auto"``: elements of gathered weights that fit in the
        free HBM left after the shards, minus an activation reserve (max(48 GiB, 25% of the
        device)).  On MI355X (288 GB) that holds one full gathered copy (keep) of Llama-2-7B at
        any world size and of Llama-2-70B from 8 ranks.  Unlimited off-GPU."""
        if self.env.device.type != "cuda":
            return 1 << 62
        from .memory_plan import live_budget_elems

        free, total = torch.cuda.mem_get_info(self.env.device)
        # blocks the caching allocator holds but no tensor uses (the full weights just sharded)
        free += torch.cuda.memory_reserved(self.env.device) - torch.cuda.memory_allocated(
            self.env.device)
        return live_budget_elems(free, total, elem_bytes)

    def stats(self) -> Dict:
        return dict(schedule=self.schedule, world=self.world, units=len(self.units),
                    total_numel=self.total_numel, max_live=self.max_live, depth=self.depth,
                    reason=self.schedule_reason,
                    pool_size=self.pool_size, turn_keep=self.turn_keep,
                    resident_units=sum(1 for u in self.units if u.resident and u.params),
                    resident_numel=self.resident_numel,
                    transposed_bwd_units=sum(1 for u in self.units if u.shard_t is not None),
                    pool_overflows=self.pool_overflows, separate_group=self.group is not None,
                    offload=self.offload)

    def pending_alloc_bytes(self) -> int:
        """HBM this coordinator will still allocate at the first micro-steps: resident units not
        gathered yet, their planned W^T copies, ring buffers not created yet (a memory estimate
        made right after engine init -- e.g. ``--gradient_checkpointing auto`` -- must count
        them: under ``keep`` that is a whole model copy plus W^T)."""
        if self.identity:
            return 0
        n = 0
        for u in self.units:
            if not u.params:
                continue
            isz = u.dtype.itemsize
            if u.resident and u.buf is None:
                n += u.padded * isz
            if u.tn and u.wt_buf is None:
                n += u.wt_numel * isz
        isz = units_dtype_bytes(self.units)
        n += max(0, self.pool_size - self._pool_alloc) * self.max_unit * isz
        return n

    # ---- buffers ----------------------------------------------------------------------------
    def _buffer(self, u: _Unit) -> torch.Tensor:
        if not self.ring or u.resident:
            if u.buf is None:
                u.buf = torch.empty(u.padded, dtype=u.dtype, device=self.device)
            return u.buf
        free = self._pool.setdefault(u.dtype, [])
        if free:
            buf = free.pop()
        else:
            if self._pool_alloc >= self.pool_size:
                self.pool_overflows += 1  # schedule bug or a model whose units re-enter
            self._pool_alloc += 1
            buf = torch.empty(self.max_unit, dtype=u.dtype, device=self.device)
        u.buf = buf
        return buf

    def _pool_free(self, dtype) -> bool:
        return bool(self._pool.get(dtype)) or self._pool_alloc < self.pool_size

    def _copy_stream(self):
        if self._cstream is None:
            self._cstream = torch.cuda.Stream(device=self.device)
        return self._cstream

    def _stage(self, shard: torch.Tensor) -> tuple:
        """Next device staging buffer of the offload ring (depth + 1 entries)."""
        n = self.depth + 1
        if not self._staging:
            self._staging = [None] * n
            self._staging_work = [None] * n
        k = self._staging_i % n
        self._staging_i += 1
        st = self._staging[k]
        if st is None or st.numel() < shard.numel():
            st = self._staging[k] = torch.empty(max(shard.numel(), self.max_unit // self.world),
                                                dtype=shard.dtype, device=self.device)
        return k, st[:shard.numel()]

    # ---- gather / bind / release ------------------------------------------------------------
    def _issue(self, i: int):
        """Gather unit i (and the units it shares parameters with) into its buffer."""
        if self.identity or i < 0 or i > self.last:
            return
        u = self.units[i]
        for d in u.deps:
            self._issue(d)
        if not u.params or u.state != "empty":
            return
        buf = self._buffer(u)
        if self.poison:  # race detector: stale reads of this buffer now see NaN
            buf.fill_(float("nan"))
        # the backward of a ring unit gathers its transposed shard (TN input-gradient GEMMs
        # straight from the buffer) unless a recompute needs the forward layout
        t = u.shard_t is not None and self._in_bwd and not self._bwd_needs_w()
        u.layout = "wt" if t else "w"
        shard, n = (u.shard_t, u.padded_t) if t else (u.shard, u.padded)
        if self.offload and buf.is_cuda:
            u.work = self._issue_offloaded(u, buf)
        elif self.local:
            u.work = _LocalGather(buf, shard)
        else:
            u.work = dist.all_gather_into_tensor(buf[:n], shard, group=self.group,
                                                 async_op=True)
        self.gathered_bytes += n * buf.element_size()
        self.gathers_t += int(t)
        self.gathers += 1
        u.state = "inflight"
        if u.tn:
            self._transpose_after_gather(u)

    def _issue_offloaded(self, u: _Unit, buf: torch.Tensor):
        """H2D copy of the pinned shard and the gather, both on the copy stream: ordered after
        the compute that last read ``buf`` (wait_stream at issue), never blocking compute."""
        cs = self._copy_stream()
        cs.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cs):
            if self.local:
                buf[:u.shard.numel()].copy_(u.shard, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cs)
                return _EventWork(ev)
            k, st = self._stage(u.shard)
            prev = self._staging_work[k]
            if prev is not None:
                prev.wait()   # the gather that last read this staging buffer is done
            st.copy_(u.shard, non_blocking=True)
            work = dist.all_gather_into_tensor(buf[:u.padded], st, group=self.group,
                                               async_op=True)
            self._staging_work[k] = work
            return work

    def _transpose_after_gather(self, u: _Unit):
        """On a side stream: wait for the gather, write W^T of the unit's projections (for the
        backward's TN input-gradient GEMMs).  The compute stream waits on the event only when it
        binds the unit."""
        from ..ops.transpose import transpose_2d

        cur = torch.cuda.current_stream(self.device)
        if self._tstream is None:
            self._tstream = torch.cuda.Stream(device=self.device)
        side = self._tstream
        if u.wt_buf is None:
            u.wt_buf = torch.empty(u.wt_numel, dtype=u.dtype, device=self.device)
        side.wait_stream(cur)      # earlier readers of this W^T are done
        with torch.cuda.stream(side):
            u.work.wait()          # side stream waits on the collective
            full, wt = u.buf, u.wt_buf
            for k, off, wt_off in u.tn:
                rows, cols = u.params[k]._zero_shape
                kp = getattr(u.params[k], "_lumen_fold_kp", 0)
                src = full[off:off + rows * (cols + kp)].view(rows, cols + kp)[:, :cols]
                transpose_2d(src, out=wt[wt_off:wt_off + rows * cols].view(cols, rows))
            ev = torch.cuda.Event()
            ev.record(side)
        u.wt_event = ev

    def restrict_transposed_gathers(self, params: Sequence[nn.Parameter]) -> int:
        """Keep the transposed backward shards only of units whose every weight belongs to a
        linear that runs its input gradient in the TN form (``transpose_bwd``): any other would
        need the forward layout in the backward.  Returns the units that keep them."""
        ok = {id(p) for p in params}
        n = 0
        for u in self.units:
            if u.shard_t is None:
                continue
            if all(id(p) in ok for p in u.params):
                n += 1
            else:
                u.shard_t, u.padded_t = None, 0
        return n

    def enable_transposes(self, params: Sequence[nn.Parameter]) -> int:
        """Keep W^T of these gathered weights next to the gathered buffer (resident units of
        keep / hybrid, when HBM allows: one more copy of the projections, written once).
        Returns the number of weights covered."""
        if self.device.type != "cuda" or not any(u.resident for u in self.units):
            return 0
        want = {id(p) for p in params}
        need = 0
        plan = []
        for u in self.units:
            if not u.resident:
                continue
            tn, o, wo = [], 0, 0
            for k, p in enumerate(u.params):
                shape = p._zero_shape
                n = math.prod(shape)
                if (id(p) in want and len(shape) == 2 and shape[0] % 8 == 0
                        and shape[1] % 8 == 0 and p.dtype in (torch.bfloat16, torch.float16)):
                    tn.append((k, o, wo))
                    wo += n
                o += _store_numel(p)
            plan.append((u, tn, wo))
            need += wo * (u.dtype.itemsize if u.dtype is not None else 2)
        free, total = torch.cuda.mem_get_info(self.device)
        # blocks the caching allocator holds but no tensor uses count as free (as in the live
        # budget): after sharding it still caches the full weights' storage
        free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
        gathered = sum(u.padded * u.dtype.itemsize for u in self.units
                       if u.params and u.buf is None and u.resident)
        gathered += self.pool_size * self.max_unit * units_dtype_bytes(self.units)
        from .memory_plan import transposes_fit

        if not transposes_fit(need, gathered, free, total):
            return 0
        n = 0
        for u, tn, wo in plan:
            u.tn, u.wt_numel = tn, wo
            n += len(tn)
            self.transposed_numel += wo
        return n

    @staticmethod
    def _bind_views(u: _Unit, full: torch.Tensor):
        o = 0
        for p in u.params:
            shape = p._zero_shape
            n = _store_numel(p)
            kp = getattr(p, "_lumen_fold_kp", 0)
            if kp:  # [N, K + KP] storage rows, the parameter is the [N, K] view
                p.data = full[o:o + n].view(shape[0], shape[1] + kp)[:, :shape[1]]
            else:
                p.data = full[o:o + n].view(shape)
            o += n

    def _wait_work(self, work):
        if not self.track_waits:
            work.wait()
            return
        if self.device.type == "cuda":
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            work.wait()
            e1.record()
            self._wait_events.append((e0, e1))
        else:
            t = time.perf_counter()
            work.wait()
            self._wait_host_s += time.perf_counter() - t

    def pop_exposed_wait_ms(self) -> float:
        """GPU time the compute stream spent blocked on gathers since the last call (call after
        a device synchronize)."""
        ms = sum(a.elapsed_time(b) for a, b in self._wait_events) + self._wait_host_s * 1e3
        self._wait_events.clear()
        self._wait_host_s = 0.0
        return ms

    def _wait(self, i: int):
        """Make unit i's params view its gathered buffer."""
        if self.identity:
            return
        u = self.units[i]
        for d in u.deps:
            self._wait(d)
        if not u.params:
            return
        if u.state == "empty":
            self._issue(i)
        if u.state == "inflight":
            self._wait_work(u.work)
            u.work = None
            u.state = "ready"
        if not u.bound and u.layout == "wt":
            # backward-only binding: W^T views for the TN input-gradient GEMMs; the forward
            # layout is absent (an accidental forward use fails on the empty weight)
            o = 0
            for p in u.params:
                rows, cols = p._zero_shape
                p.data = torch.empty(0, dtype=u.dtype, device=p.device)
                p._lumen_wt = u.buf[o:o + rows * cols].view(cols, rows)
                o += rows * cols
            u.bound = True
        if not u.bound:
            self._bind_views(u, u.buf)
            for lin in u.folds:  # freshly gathered: the adapter tail is refilled from lora_B
                lin.invalidate_fold_tail()
            if u.tn:
                if u.wt_event is not None:
                    torch.cuda.current_stream(self.device).wait_event(u.wt_event)
                    u.wt_event = None
                for k, off, wt_off in u.tn:
                    rows, cols = u.params[k]._zero_shape
                    u.params[k]._lumen_wt = u.wt_buf[wt_off:wt_off + rows * cols].view(cols, rows)
            u.bound = True

    def _unbind(self, u: _Unit):
        if u.bound:
            for p in u.params:
                p.data = torch.empty(0, dtype=u.dtype, device=p.device)
                p._lumen_wt = None
            u.bound = False

    def _release(self, i: int):
        """Drop unit i's contents (release schedule: the buffer returns to the ring; reuse is
        stream-ordered because the next gather is issued after this point)."""
        if self.identity or i < 0 or i > self.last:
            return
        u = self.units[i]
        if not u.params:
            return
        if u.resident:
            return  # keep / hybrid resident unit: gathered once, frozen, never stale
        if u.state == "inflight":
            u.work.wait()
            u.work = None
        self._unbind(u)
        if self.ring and u.buf is not None:
            self._pool.setdefault(u.dtype, []).append(u.buf)
            u.buf = None
        u.state = "empty"

    def _prefetch(self, i: int):
        """release: gather unit i ahead of use if a ring buffer is free (never grows the ring)."""
        if i < 0 or i > self.last:
            return
        u = self.units[i]
        if not u.params or u.state != "empty":
            return
        if self.ring and not u.resident and not self._pool_free(u.dtype):
            return
        self._issue(i)

    def _ahead(self, i: int, step: int, lo: int = 0):
        """The ``depth`` units to prefetch after unit i in direction ``step`` (>= lo).  Resident
        units of a hybrid schedule do not count: the look-ahead is over ring units, so a
        re-gathered unit's all-gather starts while the resident units before it compute."""
        j, n = i + step, 0
        while lo <= j <= self.last and n < self.depth:
            u = self.units[j]
            if not (self.ring and u.resident):
                yield j
                n += 1
            j += step

    # ---- model hooks ------------------------------------------------------------------------
    def _bwd_needs_w(self) -> bool:
        """Activation recompute re-runs forward GEMMs inside the backward: W, not W^T."""
        v = getattr(self.model, "gradient_checkpointing", False)
        return v not in (False, None, "none")

    def begin_micro_step(self):
        self._bwd_seen.clear()
        self._in_step = True
        self._in_bwd = False
        if self.identity:
            return
        for i in self._ahead(-1, 1):
            self._prefetch(i)          # (keep: no-op once the units are resident)

    def pre_forward(self, i: int):
        if i == 0 and not self._in_step:
            self.begin_micro_step()
        if self.identity:
            return
        self._wait(i)
        for j in self._ahead(i, 1):
            self._prefetch(j)

    def post_forward(self, i: int, out):
        # release / hybrid: the head (last) and the ``turn_keep`` units before it are consumed
        # by the backward right after the turn and stay live; every other ring unit is freed
        if self.ring and i < self.last - self.turn_keep:
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
            torch.autograd.Variable._execution_engine.queue_callback(self.end_micro_step)
        self._bwd_seen.add(i)
        if self.identity:
            return
        self._in_bwd = True
        if self.ring:
            self._release(i + 1)
        self._wait(i)
        if self.ring:
            for j in self._ahead(i, -1, lo=1):
                self._prefetch(j)  # unit 0 (embedding) has no backward

    def end_micro_step(self):
        """After the backward (or a no-grad forward): nothing of this micro-step is read any
        more.  Idempotent (the autograd callback and the engine both call it)."""
        if not self._in_step:
            return
        self._in_step = False
        self._in_bwd = False
        if self.identity or self.keep:
            return  # keep: the gathered frozen weights stay resident
        for i in range(self.last + 1):
            self._release(i)   # (hybrid: resident units stay)

    def gather_all_full(self) -> None:
        """Materialise every unit (checkpoint save with gather_16bit_weights_on_model_save).
        The release ring grows for this (the save is outside the step loop)."""
        self._in_bwd = False
        for i in range(self.last + 1):
            if self.units[i].layout == "wt":
                self._release(i)
            self._issue(i)
            self._wait(i)

    def release_all(self):
        for i in range(self.last + 1):
            self._release(i)
        self._in_step = False
        for free in self._pool.values():  # gather_all_full grew the ring: shrink it back
            while self._pool_alloc > self.pool_size and free:
                free.pop()
                self._pool_alloc -= 1

    def drain(self):
        """Complete every in-flight gather: before process-group teardown."""
        for u in self.units:
            if u.work is not None:
                u.work.wait()
                u.work = None
                u.state = "ready"


def _t_eligible(u: _Unit) -> bool:
    """A unit whose backward can run on a transposed gather: every parameter a 16-bit 2-D
    projection weight with 8-aligned dims (the TN input-gradient GEMM's operand)."""
    return all(len(p._zero_shape) == 2 and p._zero_shape[0] % 8 == 0
               and p._zero_shape[1] % 8 == 0 and p.dtype in (torch.bfloat16, torch.float16)
               for p in u.params)


def units_dtype_bytes(units: Sequence[_Unit]) -> int:
    return max((u.dtype.itemsize for u in units if u.params), default=2)


def _store_numel(p) -> int:
    """Elements of p in the unit's flat storage ([N, K + KP] rows for a LoRA-folded weight)."""
    kp = getattr(p, "_lumen_fold_kp", 0)
    shape = getattr(p, "_zero_shape", tuple(p.shape))
    return shape[0] * (shape[1] + kp) if kp else math.prod(shape)


def _stored(t: torch.Tensor, kp: int) -> torch.Tensor:
    return torch.nn.functional.pad(t, (0, kp)) if kp else t


def _mark_fold_weights(model: nn.Module) -> Dict[int, nn.Module]:
    """Linears whose LoRA forward will run K-extended: tag their frozen weight with the tail
    width (``_lumen_fold_kp``) so the partitioned layout reserves it.  {id(weight): linear}"""
    out: Dict[int, nn.Module] = {}
    for m in model.modules():
        f = getattr(m, "fold_ext", None)
        if f is not None and f(static=True):
            m.weight._lumen_fold_kp = f(static=True)
            out[id(m.weight)] = m
    return out


def mark_zero_shapes(model: nn.Module):
    for p in model.parameters():
        if not hasattr(p, "_zero_shape"):
            p._zero_shape = tuple(p.shape)
