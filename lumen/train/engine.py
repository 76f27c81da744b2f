"""Training engine: ZeRO stage 0-3 data parallel step over a (LoRA-)model.

Replaces what the reference gets from ``deepspeed.initialize`` inside HF Trainer
(reference CS3/CS4: training/train.ipynb:780-806, configs/ds_config_zero*.json):
forward / backward with loss scaling and gradient accumulation, ZeRO gradient reduction,
global-norm clipping, AdamW (GPU fused kernel, or CPU when offloaded), WarmupLR, ZeRO-3
parameter coordination, and sharded state for checkpoints.

Engine API (DeepSpeed-like):
    loss = engine.forward(batch)          # batch: dict(input_ids, labels, n_valid) on device
    engine.backward(loss)                 # scales for fp16 + grad accumulation, reduces (stage 2/3)
    stepped = engine.step()               # at the accumulation boundary: reduce/clip/update/gather
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..parallel.dist import DistEnv
from ..parallel.zero import (AsyncOffloadStep, DynamicLossScaler, FlatTrainable,
                             ParamCoordinator, ShardAdamW, grad_norm_sq, overlap_bucket_numel)
from .config import DSConfig, warmup_lr


class Timers:
    """Per-phase wall-clock breakdown (DeepSpeed ``wall_clock_breakdown`` semantics)."""

    def __init__(self, enabled: bool, device):
        self.enabled = enabled
        self.device = device
        self.acc: Dict[str, float] = {}
        self._t: Dict[str, float] = {}

    def start(self, k):
        if self.enabled:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self._t[k] = time.perf_counter()

    def stop(self, k):
        if self.enabled:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.acc[k] = self.acc.get(k, 0.0) + time.perf_counter() - self._t.pop(k)

    def pop(self) -> Dict[str, float]:
        a, self.acc = self.acc, {}
        return a


class ZeroEngine:
    def __init__(self, model: nn.Module, cfg: DSConfig, env: DistEnv):
        self.model = model
        self.cfg = cfg
        self.env = env
        self.device = env.device
        self.stage = cfg.stage
        W = env.world_size
        self.sharded = W > 1 and self.stage >= 1
        self.micro_step = 0
        self.global_step = 0
        self._scaler_skipped = 0
        self.last_grad_norm: Optional[torch.Tensor] = None
        self.timers = Timers(cfg.wall_clock_breakdown, self.device)

        trainable = [p for p in model.parameters() if p.requires_grad]
        if not trainable:
            raise ValueError("model has no trainable parameters")
        # ZeRO-3: partition frozen weights first (trainable adapters stay persistent).  At world
        # size 1 the one-rank partition is the whole unit ("identity" schedule: no gathers);
        # LUMEN_ZERO3_SINGLE=1 forces per-step materialisation there (a side-stream copy with
        # RCCL's stream semantics) to run the gather schedules on a single-GPU box.
        self.coordinator: Optional[ParamCoordinator] = None
        self.gather_group = None
        single = os.environ.get("LUMEN_ZERO3_SINGLE", "0") == "1"
        if self.stage >= 3:
            if W > 1 and dist.is_initialized() and os.environ.get(
                    "LUMEN_ZERO3_SHARED_GROUP", "0") != "1":
                # weight gathers on their own communicator (own RCCL stream): gradient
                # reduce-scatters / norm / publish on the default group never queue behind them
                self.gather_group = dist.new_group(ranks=list(range(W)))
            self.coordinator = ParamCoordinator(
                model, env, cfg.stage3_param_persistence_threshold,
                cfg.stage3_max_live_parameters, cfg.stage3_prefetch_bucket_size,
                offload_param=cfg.offload_param == "cpu", pin_memory=cfg.offload_param_pin,
                schedule=os.environ.get("LUMEN_ZERO3_SCHEDULE") or None,
                group=self.gather_group, max_reuse_distance=cfg.stage3_max_reuse_distance,
                force_partition=single)
            model.coordinator = self.coordinator
            if self.gather_group is not None and self.coordinator.keep:
                # keep gathers each unit once (warm-up): a second communicator would buy no
                # overlap, only a second RCCL communicator per GPU (never initialised: RCCL
                # communicators are created at their first collective)
                self.coordinator.group = None
                self.gather_group = None
            if env.is_main:  # stderr: bench.py's stdout is exactly one JSON line
                import sys

                c = self.coordinator
                print(f"[lumen] ZeRO-3 schedule '{c.schedule}': {c.schedule_reason}",
                      file=sys.stderr, flush=True)
        if self.device.type == "cuda":
            from ..models.layers import configure_backward_layout

            configure_backward_layout(model)  # TN input-gradient GEMMs for persistent weights
            if self.coordinator is not None:
                # ring units' backward gathers their transposed shards: only for linears that
                # take the TN input-gradient GEMM
                from ..models.layers import Linear

                self.coordinator.restrict_transposed_gathers(
                    [m.weight for m in model.modules() if isinstance(m, Linear)
                     and m.transpose_bwd])
            # ... and for resident (keep / hybrid) gathered ones: W^T written once, on a side
            # stream right after the unit's first gather, when HBM allows (ring units are
            # re-gathered every use and keep the on-the-fly q|k|v / down transposes,
            # Linear.transpose_gathered)
            if self.coordinator is not None and (self.coordinator.keep
                                                 or self.coordinator.schedule == "hybrid"):
                from ..models.layers import Linear

                self.coordinator.enable_transposes(
                    [m.weight for m in model.modules() if isinstance(m, Linear)
                     and m.transpose_bwd and getattr(m.weight, "_lumen_gathered", False)])
        bucket = cfg.reduce_bucket_size if self.stage >= 1 else int(2.5e7)
        bucket = overlap_bucket_numel(bucket, W, self.sharded and self.stage >= 2
                                      and cfg.overlap_comm)
        self.flat = FlatTrainable(trainable, env, max(bucket, 1), self.device)
        # broadcast adapter init from rank 0 (only the trainable 32 MiB, not 13.5 GB)
        if W > 1:
            dist.broadcast(self.flat.param, src=0)
        n_opt = self.flat.shard_numel if self.sharded else self.flat.numel
        self.opt = ShardAdamW(n_opt, self.device, cfg.betas, cfg.eps, cfg.weight_decay,
                              offload=cfg.offload_optimizer == "cpu",
                              pin_memory=cfg.offload_optimizer_pin)
        with torch.no_grad():
            src = self.flat.gather_shard(self.flat.param) if self.sharded else self.flat.param
            self.opt.master.copy_(src)
        # stage 2/3 accumulate reduced shards across micro-steps
        self.grad_shard = (torch.zeros(self.flat.shard_numel, dtype=torch.float32,
                                       device=self.device) if self.sharded else None)
        self._tmp_shard = (torch.zeros_like(self.grad_shard) if self.sharded and self.stage >= 2
                           else None)
        self.scaler = None
        if cfg.dtype == "fp16":
            self.scaler = DynamicLossScaler(2.0 ** cfg.initial_scale_power, cfg.loss_scale_window,
                                            cfg.hysteresis, cfg.min_loss_scale, cfg.loss_scale)
        # GPU: LR warm-up, Adam bias correction and the fp16 loss scaler run on the device from
        # the applied-step counter (no host sync per step, bf16 or fp16); host logic otherwise
        self.device_sched = self.opt.configure_schedule(
            cfg.warmup_min_lr, cfg.warmup_max_lr, cfg.warmup_num_steps,
            cfg.warmup_type == "linear", W, self.scaler,
            cfg.decay_total_steps if cfg.lr_schedule in self._DECAYING else 0,
            self._DECAYING.index(cfg.lr_schedule) if cfg.lr_schedule in self._DECAYING else 0,
            cfg.cos_min_ratio)
        self._norm_buf = torch.zeros(1, dtype=torch.float32, device=self.device)
        self._k = 1  # accumulation micro-steps fused into the current forward / backward
        # ZeRO-Offload optimizer: the CPU step overlaps the next forward (exact semantics)
        self.async_off: Optional[AsyncOffloadStep] = None
        if (self.opt.offload and self.device.type == "cuda" and not self.device_sched
                and os.environ.get("LUMEN_OFFLOAD_ASYNC", "1") != "0"):
            from ..ops._native import native

            if native() is not None:
                self.async_off = AsyncOffloadStep(self.opt, self.flat, self.device, self.sharded)
                self.async_off.map_units(model)
                model.unit_gate = self.async_off.gate
        from ..models.layers import FoldTails

        self.fold_tails = FoldTails(model) if self.device.type == "cuda" else None
        self._gscale = torch.ones(1, dtype=torch.float32, device=self.device)
        self._works: List = []
        for prm in trainable:  # .grad is a view of flat.grad: kernels may accumulate into it
            prm._lumen_direct_grad = True
        if self.sharded and self.stage >= 2 and cfg.overlap_comm:
            self._install_bucket_hooks()

    # ----------------------------------------------------------------------------------------
    @property
    def loss_scale(self) -> float:
        """Current loss scale (device path: reads the device state, syncs)."""
        if self.device_sched and self.scaler is not None:
            return float(self.opt.state[2].item())
        return self.scaler.scale if self.scaler else 1.0

    @property
    def last_lr(self) -> float:
        """LR of the last optimizer step: DeepSpeed WarmupLR indexed by APPLIED steps (an
        overflow-skipped step does not advance the scheduler)."""
        applied = self.opt.step_count
        return warmup_lr(max(applied - 1, 0), self.cfg) if applied else warmup_lr(0, self.cfg)

    # decaying schedules, by the device kernel's decay_kind
    _DECAYING = ("hf_linear", "warmup_decay", "warmup_cosine")

    def set_total_steps(self, n: int) -> None:
        """Run length for a decaying schedule (HF linear: no DeepSpeed config; DeepSpeed
        WarmupDecayLR / WarmupCosineLR with total_num_steps "auto")."""
        if self.cfg.lr_schedule not in self._DECAYING or (
                self.cfg.lr_schedule != "hf_linear" and self.cfg.decay_total_steps > 0):
            return
        self.cfg.decay_total_steps = int(n)
        if self.device_sched:
            self.opt.sched[9] = float(n)

    def is_boundary(self) -> bool:
        return (self.micro_step + self._k) % self.cfg.grad_accum == 0

    def lr(self) -> float:
        """LR for the next update (host path): WarmupLR at the applied-step count."""
        return warmup_lr(self.opt.step_count, self.cfg)

    # ---- stage 2/3: reduce-scatter buckets as soon as backward finished them ----------------
    def _install_bucket_hooks(self):
        for b in self.flat.buckets:
            for p in b.params:
                hook = self._make_ready_hook(b)
                p.register_post_accumulate_grad_hook(hook)
                # kernels that accumulate into .grad directly (lora_bwd_native) report here
                p._lumen_grad_ready = hook

    def _make_ready_hook(self, b):
        def hook(p):
            b.ready += 1
            if b.ready == len(b.params):
                self._reduce_bucket(b, async_op=True)
        return hook

    def _reduce_bucket(self, b, async_op: bool):
        out = self.flat.shard_view(self._tmp_shard, b)
        work = dist.reduce_scatter_tensor(out, self.flat.grad[b.off:b.off + b.size],
                                          async_op=async_op)
        b.work = work

    # ----------------------------------------------------------------------------------------
    def forward(self, batch: Dict) -> torch.Tensor:
        """``batch["micro_steps"]`` = k > 1: the batch is k accumulation micro-batches fused
        into one (the trainer does this when they hold equal valid-token counts, so the fused
        mean loss IS the mean of their means): backward scales by k / grad_accum and the step
        counts k micro-steps."""
        self.timers.start("fwd")
        self._k = int(batch.get("micro_steps", 1))
        fp16_dev = self.device_sched and self.scaler is not None
        if fp16_dev:
            # the fused LM-head CE writes dlogits already multiplied by the scale the backward
            # will apply (device scalar: no host read of the loss scale)
            from ..ops import loss as loss_ops

            torch.div(self.opt.state[2:3], self.cfg.grad_accum / self._k, out=self._gscale)
            loss_ops.GRAD_SCALE_HINT[0] = self._gscale
        try:
            kw = {"cu_seqlens": batch["cu_seqlens"]} if batch.get("cu_seqlens") is not None else {}
            loss = self.model(batch["input_ids"], batch["labels"], batch.get("n_valid"),
                              batch.get("pos"), **kw)
        finally:
            if fp16_dev:
                loss_ops.GRAD_SCALE_HINT[0] = None
        self.timers.stop("fwd")
        return loss

    __call__ = forward

    def backward(self, loss: torch.Tensor):
        self.timers.start("bwd")
        if self.async_off is not None:
            self.async_off.before_backward()
        if self.device_sched and self.scaler is not None:
            # fp16: scale by the device loss scale / accum (no host read of it); the same tensor
            # the forward handed the CE kernel as its gradient-scale hint
            (loss * self._gscale[0]).backward()
        else:
            scale = self.loss_scale * self._k / self.cfg.grad_accum
            (loss * scale if scale != 1.0 else loss).backward()
        if self.coordinator is not None:
            self.coordinator.end_micro_step()
        if self.sharded and self.stage >= 2:
            # every bucket reduce-scattered this micro-step (hooks launched them during backward)
            for b in self.flat.buckets:
                if b.work is None:
                    self._reduce_bucket(b, async_op=True)
            for b in self.flat.buckets:
                b.work.wait()
                b.work = None
                b.ready = 0
            self.grad_shard.add_(self._tmp_shard)
            self.flat.grad.zero_()
        self.timers.stop("bwd")

    @torch.no_grad()
    def step(self) -> bool:
        """Call after every backward; updates only at the accumulation boundary."""
        boundary = self.is_boundary()
        self.micro_step += self._k
        self._k = 1
        if not boundary:
            return False
        self.timers.start("step")
        W = self.env.world_size
        if not self.sharded:
            if W > 1:  # stage 0: plain data parallel all-reduce
                for b in self.flat.buckets:
                    dist.all_reduce(self.flat.grad[b.off:b.off + b.size])
            grad = self.flat.grad
        elif self.stage == 1:
            for b in self.flat.buckets:
                dist.reduce_scatter_tensor(self.flat.shard_view(self.grad_shard, b),
                                           self.flat.grad[b.off:b.off + b.size])
            grad = self.grad_shard
        else:
            grad = self.grad_shard
        # global grad norm (of the raw summed grads) -> device scalar, all-reduced over shards
        self._norm_buf.zero_()
        grad_norm_sq(grad, self._norm_buf)
        if self.sharded:
            dist.all_reduce(self._norm_buf)
        # grads are sums over ranks of (loss * scale / accum) gradients
        if self.device_sched:
            # one kernel: unscale, clip, skip-on-overflow, bias correction, WarmupLR and the
            # loss-scaler update all read / advance device state -- no host sync
            self.last_grad_norm = self._norm_buf.sqrt() / (self.opt.state[2] * W)
            self.opt.step(grad, 0.0, 0.0, self._norm_buf, self.cfg.gradient_clipping)
            self._publish_params()   # a skipped step publishes unchanged values
        else:
            inv_scale = 1.0 / (self.loss_scale * W)
            lr = self.lr()
            overflow = False
            if self.scaler is not None:
                nsq = float(self._norm_buf.item())
                overflow = not math.isfinite(nsq)
                self.scaler.update(overflow)
            launched = None
            if overflow:
                self._scaler_skipped += 1
            elif self.async_off is not None:
                hp = self.opt.host_coef(self._norm_buf, inv_scale, self.cfg.gradient_clipping)
                if hp is not None:  # None: non-finite norm, counted as skipped
                    self.async_off.launch(grad, lr, *hp)
                    self.flat.mark_updated()  # params land under the next forward's unit gates
                    launched = grad  # zeroed by the offload stream after its D2H
            else:
                self.opt.step(grad, lr, inv_scale, self._norm_buf, self.cfg.gradient_clipping)
                self._publish_params()
            self.last_grad_norm = self._norm_buf.sqrt() * inv_scale
            if launched is not None:
                if launched is not self.flat.grad:
                    self.flat.grad.zero_()
                self.global_step += 1
                self.timers.stop("step")
                return True
        self.flat.grad.zero_()
        if self.grad_shard is not None:
            self.grad_shard.zero_()
        self.global_step += 1
        self.timers.stop("step")
        return True

    def _publish_params(self):
        """Write the updated master shard back to the model's flat params (+ all-gather)."""
        master = self.opt.master
        if master.device != self.device:
            master = master.to(self.device, non_blocking=True)
        self.flat.mark_updated()
        if not self.sharded:
            self.flat.param.copy_(master)
        else:
            for b in self.flat.buckets:
                dist.all_gather_into_tensor(self.flat.param[b.off:b.off + b.size],
                                            self.flat.shard_view(master, b))
        if self.fold_tails is not None:
            self.fold_tails.refresh()  # every folded linear's [s B] tail, one launch

    def _scaler_state(self):
        if self.scaler is None:
            return None
        if self.device_sched:
            sc, hy, it, lo = self.opt.state[2:6].tolist()
            return dict(scale=sc, cur_hysteresis=int(hy), iter=int(it), last_overflow_iter=int(lo))
        return self.scaler.state_dict()

    @property
    def skipped_steps(self) -> int:
        """Steps skipped for a non-finite gradient: fp16 overflows seen by the loss scaler plus
        bf16 NaN/Inf steps the fused AdamW kernel skipped on the device (reading that syncs)."""
        return self._scaler_skipped + self.opt.skipped

    def sync_params(self) -> None:
        """Finish a pending asynchronous (offloaded) optimizer step: params current."""
        if self.async_off is not None:
            self.async_off.finish()

    def close(self):
        """Complete in-flight ZeRO-3 gathers (prefetches issued ahead of their use) so the process
        groups can be torn down cleanly."""
        self.sync_params()
        if self.coordinator is not None:
            self.coordinator.drain()

    # ---- checkpoint state ----------------------------------------------------------------------
    def state_dict(self) -> Dict:
        from .reshard import engine_layout

        self.sync_params()

        return dict(optimizer=self.opt.state_dict(), global_step=self.global_step,
                    micro_step=self.micro_step, skipped_steps=self.skipped_steps,
                    scaler=self._scaler_state(),
                    stage=self.stage, world_size=self.env.world_size,
                    shard_numel=self.opt.master.numel(), layout=engine_layout(self))

    def load_state_dict(self, d: Dict):
        self.sync_params()
        if d["shard_numel"] != self.opt.master.numel():
            raise ValueError("checkpoint shard layout does not match (world size / stage changed): "
                             "load it through lumen.train.reshard.load_engine_state")
        self.opt.load_state_dict(d["optimizer"])
        self.global_step = d["global_step"]
        self.micro_step = d["micro_step"]
        self._scaler_skipped = d.get("skipped_steps", 0)
        if self.scaler and d.get("scaler"):
            self.scaler.load_state_dict(d["scaler"])
            if self.device_sched:
                sc = d["scaler"]
                self.opt.state[2:6] = torch.tensor(
                    [sc["scale"], sc["cur_hysteresis"], sc["iter"], sc["last_overflow_iter"]],
                    dtype=torch.float32)
        with torch.no_grad():
            self._publish_params()
