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
* ZeRO-3 partitions the frozen base weights per unit (embedding, each decoder layer, head):
  see lumen/parallel/zero3.py (own RCCL communicator for the weight gathers, keep (gathered once,
  resident) / release / identity schedules, offloaded shards on a copy stream).
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


# Gradient buckets of the overlapped (ZeRO-2/3) reduce-scatter (opt-in, LUMEN_DP_BUCKET_MB > 0).
# A LoRA-sized trainable set fits one DeepSpeed-sized bucket (16.8 M elements against
# reduce_bucket_size 5e7), and that single reduce-scatter can only start once the whole
# backward has finished.  Buckets of e.g. 16 MiB of fp32 gradients let every
# bucket but the last reduce under the remaining layers' backward.
# Off by default, because it is unmeasured on an 8-GPU node:
# * on this chip, concurrent kernels have so far cost the compute kernel more than they hid
#   (profiles/r5_mlp_overlap: a tail GEMM beside the SwiGLU ran 2x longer);
# * an RCCL kernel holding CUs during a one-wave backward GEMM can push that GEMM's tiles into a
#   second wave;
# * the single reduce-scatter it would hide is ~0.3 % of the step.
# The bench records dp_grad_buckets, and extra.comm records the reduce-scatter size sweep, so
# the node's own numbers can decide this.
DP_BUCKET_MB = float(os.environ.get("LUMEN_DP_BUCKET_MB", "0"))


def overlap_bucket_numel(cfg_numel: int, world: int, overlapped: bool,
                         cap_mb: Optional[float] = None) -> int:
    """Bucket size (fp32 elements) for the flat gradient buffer: the config's, capped at
    ``cap_mb`` MiB when world > 1 and the reduce-scatter overlaps the backward."""
    cap_mb = DP_BUCKET_MB if cap_mb is None else cap_mb
    if world <= 1 or not overlapped or cap_mb <= 0:
        return cfg_numel
    return min(cfg_numel, max(int(cap_mb * 2**20) // 4, 1))


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

    def mark_updated(self) -> None:
        """The flat buffer was rewritten (optimizer publish): bump every parameter's autograd
        version counter.  The params are views installed with ``p.data = ...``, whose counters
        do not see writes through ``self.param`` -- and caches keyed on ``_version`` (the LoRA
        fold's [W | s B] tail, lumen.models.layers.Linear.fold_weight) must."""
        from torch.autograd.graph import increment_version

        increment_version([p for b in self.buckets for p in b.params])

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


# ZeRO-3 parameter coordinator: lumen/parallel/zero3.py (re-exported here)
from .zero3 import ParamCoordinator, mark_zero_shapes, units_dtype_bytes  # noqa: E402,F401


# ================================================================================================
# optimizer state on a shard
# ================================================================================================

class ShardAdamW:
    """AdamW over this rank's f32 shard: HIP fused kernel on GPU, C++ AVX-512 kernel when
    offloaded to CPU, torch math on CPU tensors (tests).

    On the GPU path the Adam step counter lives on the device (``state`` = [applied, skipped]):
    the kernel derives the bias corrections from it and a non-finite grad norm skips the update
    WITHOUT advancing it, so bf16 steps stay sync-free and a NaN step can never desynchronise the
    bias correction from the number of updates actually applied."""

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
        self._host_step = 0
        self._host_skipped = 0
        # device schedule state (see kernels/adamw.hip OptSched): [applied, skipped, loss scale,
        # cur hysteresis, scaler iter, last overflow iter, -, -]
        self.state = None
        self.sched: Optional[List[float]] = None
        if not offload and device.type == "cuda":
            self.state = torch.zeros(8, dtype=torch.float32, device=device)
            self.state[2] = 1.0

    def configure_schedule(self, lr_min: float, lr_max: float, warm_n: int, warm_linear: bool,
                           world: int, scaler=None, decay_total: int = 0, decay_kind: int = 0,
                           cos_min: float = 0.0) -> bool:
        """Move the LR schedule (DeepSpeed WarmupLR, or HF's linear warm-up + decay when
        ``decay_total`` > 0) and (fp16) the dynamic loss scaler onto the device.
        Returns True when the device path is active (GPU, fused kernel available)."""
        if self.state is None or not use_native(self.master):
            return False
        dyn = scaler is not None and not scaler.static
        self.sched = [lr_min, lr_max, float(warm_n), 1.0 if warm_linear else 0.0, 1.0 / world,
                      1.0 if dyn else 0.0, float(scaler.window if scaler else 1000),
                      float(scaler.hysteresis if scaler else 2),
                      float(scaler.min_scale if scaler else 1.0), float(decay_total),
                      float(decay_kind), float(cos_min)]
        st = [0.0, 0.0, float(scaler.scale) if scaler else 1.0,
              float(scaler.cur_hysteresis if scaler else 2), 0.0, -1.0, 0.0, 0.0]
        self.state.copy_(torch.tensor(st, dtype=torch.float32))
        return True

    @property
    def device_sched(self) -> bool:
        return self.sched is not None

    @property
    def step_count(self) -> int:
        """Applied updates (device counter read on the GPU path: syncs)."""
        if self.state is not None and use_native(self.master):
            return self._host_step + int(self.state[0].item())
        return self._host_step

    @property
    def skipped(self) -> int:
        if self.state is not None and use_native(self.master):
            return self._host_skipped + int(self.state[1].item())
        return self._host_skipped

    def host_coef(self, norm_sq: torch.Tensor, inv_scale: float, max_norm: float):
        """Host-path step preamble (reads the norm: syncs): (grad coefficient, bc1, bc2) with
        clipping folded in and the step counted, or None for a non-finite norm (skipped)."""
        nsq = float(norm_sq.item())
        if not math.isfinite(nsq):
            self._host_skipped += 1
            return None
        coef = inv_scale
        gn = math.sqrt(nsq) * inv_scale
        if max_norm > 0 and gn > max_norm:
            coef *= max_norm / (gn + 1e-6)
        self._host_step += 1
        t = self._host_step
        return coef, 1 - self.b1 ** t, 1 - self.b2 ** t

    def step(self, grad: torch.Tensor, lr: float, inv_scale: float,
             norm_sq: Optional[torch.Tensor], max_norm: float) -> None:
        if self.state is not None and use_native(self.master):
            # bias corrections from the device counter; with a device schedule also the LR and
            # the loss-scale unscale (then ``lr`` / ``inv_scale`` are ignored)
            sched = self.sched if self.sched is not None else [
                lr, lr, 0.0, 0.0, inv_scale, 0.0, 1000.0, 2.0, 1.0]
            if self.sched is None:
                self.state[2] = 1.0
            native().adamw(self.master, grad, self.m, self.v, None, lr, self.b1, self.b2,
                           self.eps, self.wd, 1.0, 1.0, inv_scale, norm_sq, max_norm, self.state,
                           sched)
            return
        coef = inv_scale
        if norm_sq is not None:
            nsq = float(norm_sq.item())
            if not math.isfinite(nsq):
                self._host_skipped += 1
                return
            gn = math.sqrt(nsq) * inv_scale
            if max_norm > 0 and gn > max_norm:
                coef *= max_norm / (gn + 1e-6)
        self._host_step += 1
        t = self._host_step
        bc1, bc2 = 1 - self.b1 ** t, 1 - self.b2 ** t
        p = self.master
        if self.offload:
            g = grad.to("cpu", non_blocking=False) if grad.is_cuda else grad
            C = native()
            if C is not None:
                C.cpu_adamw(p, g.contiguous(), self.m, self.v, lr, self.b1, self.b2, self.eps,
                            self.wd, bc1, bc2, coef)
            else:
                _adamw_torch(p, g, self.m, self.v, lr, self.b1, self.b2, self.eps, self.wd, bc1,
                             bc2, coef)
            return
        _adamw_torch(p, grad, self.m, self.v, lr, self.b1, self.b2, self.eps, self.wd, bc1, bc2, coef)

    def state_dict(self):
        return dict(master=self.master.cpu(), exp_avg=self.m.cpu(), exp_avg_sq=self.v.cpu(),
                    step=self.step_count, betas=(self.b1, self.b2), eps=self.eps, wd=self.wd)

    def load_state_dict(self, d):
        self.master.copy_(d["master"])
        self.m.copy_(d["exp_avg"])
        self.v.copy_(d["exp_avg_sq"])
        self._host_skipped = 0
        if self.state is not None and use_native(self.master):
            # the device counter drives bias correction (and the LR schedule): restore it there
            self._host_step = 0
            self.state[0] = float(d["step"])
            self.state[1] = 0.0
        else:
            self._host_step = int(d["step"])


class AsyncOffloadStep:
    """ZeRO-Offload optimizer step overlapped with the next forward (exact semantics: no stale
    parameters; reference ``offload_optimizer: cpu``, configs/ds_config_zero3.json:19-22).

    The step is cut into ``n_chunks`` slices of the flat shard, processed in FORWARD order (the
    flat buffer is laid out backward-first, so from its end):

    * copy stream: D2H of every gradient slice into pinned host memory (event per slice), then
      the gradient buffer is zeroed there -- the compute stream only waits for that before its
      next backward;
    * host thread: per slice, wait for its D2H, C++ AVX-512 AdamW (GIL released), H2D of the
      updated master slice into the device parameters (event per slice);
    * the model calls ``gate(unit)`` before each unit's forward: the host waits until the
      slices holding that unit's adapters are updated and the compute stream waits on their
      H2D events.  Layer 1's adapters are ready after 1/n of the CPU step; the rest of the CPU
      work runs under the forward of the layers before it.

    Sharded ranks (world > 1) update their shard the same way into a device staging shard; the
    first gate of the step joins the host thread and issues the publish all-gathers from the
    main thread (collectives stay on one thread, in program order on every rank)."""

    def __init__(self, opt: "ShardAdamW", flat: "FlatTrainable", device: torch.device,
                 sharded: bool, n_chunks: int = 16):
        import threading

        self.opt, self.flat, self.device, self.sharded = opt, flat, device, sharded
        n = opt.master.numel()
        k = max(1, min(n_chunks, n // 4096))
        step = _round_up((n + k - 1) // k, ALIGN)
        bounds = [(a, min(a + step, n)) for a in range(0, n, step)]
        self.chunks = bounds[::-1]          # forward order: the flat layout is backward-first
        self.stream = torch.cuda.Stream(device=device)
        self.g_host = torch.empty(n, dtype=torch.float32).pin_memory()
        self.dst_shard = torch.empty(n, dtype=torch.float32, device=device) if sharded else None
        self._thread: Optional[threading.Thread] = None
        self._done = [threading.Event() for _ in self.chunks]
        self._h2d: List[Optional[torch.cuda.Event]] = [None] * len(self.chunks)
        self._grad_free: Optional[torch.cuda.Event] = None
        self._err: Optional[BaseException] = None
        self.pending = False
        self.unit_chunks: Dict[int, List[int]] = {}

    def map_units(self, model: nn.Module) -> None:
        """unit index -> chunks holding its trainable parameters (world-1 flat offsets)."""
        if self.sharded or not hasattr(model, "zero_units"):
            return
        for i, mods in enumerate(model.zero_units()):
            ks = set()
            for m in mods:
                for p in m.parameters():
                    if not p.requires_grad or id(p) not in self.flat.index:
                        continue
                    _, o, n = self.flat.index[id(p)]
                    ks.update(j for j, (a, b) in enumerate(self.chunks) if a < o + n and o < b)
            self.unit_chunks[i] = sorted(ks)

    def launch(self, grad: torch.Tensor, lr: float, coef: float, bc1: float, bc2: float) -> None:
        """Start the step for an already-reduced gradient (``grad`` = the flat gradient at world
        1, the reduced shard otherwise).  Returns at once."""
        import threading

        self.join()
        o = self.opt
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        d2h = []
        with torch.cuda.stream(self.stream):
            for a, b in self.chunks:
                self.g_host[a:b].copy_(grad[a:b], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
                d2h.append(ev)
            grad.zero_()
            self._grad_free = torch.cuda.Event()
            self._grad_free.record(self.stream)
        for e in self._done:
            e.clear()
        self._h2d = [None] * len(self.chunks)
        self._err = None
        dst = self.dst_shard if self.sharded else self.flat.param
        C = native()

        def work():
            try:
                torch.cuda.set_device(self.device)
                for j, (a, b) in enumerate(self.chunks):
                    d2h[j].synchronize()
                    C.cpu_adamw(o.master[a:b], self.g_host[a:b], o.m[a:b], o.v[a:b], lr, o.b1,
                                o.b2, o.eps, o.wd, bc1, bc2, coef)
                    with torch.cuda.stream(self.stream):
                        dst[a:b].copy_(o.master[a:b], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    self._h2d[j] = ev
                    self._done[j].set()
            except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
                self._err = e
                for ev in self._done:
                    ev.set()

        self.pending = True
        self._thread = threading.Thread(target=work, name="lumen-offload-adam", daemon=True)
        self._thread.start()

    def _check(self):
        if self._err is not None:
            err, self._err = self._err, None
            raise RuntimeError("async offloaded AdamW step failed") from err

    def gate(self, unit: int) -> None:
        if not self.pending:
            return
        if self.sharded or unit not in self.unit_chunks:
            self.finish()
            return
        cur = torch.cuda.current_stream(self.device)
        for j in self.unit_chunks[unit]:
            self._done[j].wait()
            self._check()
            cur.wait_event(self._h2d[j])

    def finish(self) -> None:
        """Everything of the pending step is on the device (and published when sharded)."""
        if not self.pending:
            return
        self.join()
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.stream)
        if self.sharded:
            for b in self.flat.buckets:
                dist.all_gather_into_tensor(self.flat.param[b.off:b.off + b.size],
                                            self.flat.shard_view(self.dst_shard, b))
        self.pending = False

    def join(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        self._check()

    def before_backward(self) -> None:
        """The next backward accumulates into the gradient buffer: after its zeroing."""
        if self._grad_free is not None:
            torch.cuda.current_stream(self.device).wait_event(self._grad_free)
            self._grad_free = None


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
