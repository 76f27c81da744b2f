"""Training loop (replaces the reference's HF Trainer usage).

Reference behaviour kept: per-rank sharded data, micro-batch x grad-accum, logging every
``logging_steps`` (10) optimizer steps with keys {loss, grad_norm, learning_rate, epoch}
(training/train.ipynb:339), periodic ``checkpoint-N`` saves with rotation, resume, final PEFT
export to ``{output_dir}/final`` and a metrics row (training/train_baseline.py:236-255).
Added: tokens/s and TFLOP/s, ``max_steps``, synthetic data, random init (offline).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

import torch

from ..data import (CausalLMCollator, PackedCollator, PrefetchLoader, ShardedSampler,
                    build_dataset, load_tokenizer)
from ..lora import LoraConfig, apply_lora, print_trainable_parameters, save_adapter
from ..models import build_model, get_config
from ..parallel.dist import DistEnv, agree_all, all_reduce_scalar, barrier
from ..utils.debug import StepProfiler, StepWatchdog, check_finite, maybe_inject_fault
from .checkpoint import AsyncCheckpointer, latest_checkpoint, load_checkpoint, save_checkpoint
from .config import DSConfig
from .engine import ZeroEngine


@dataclass
class TrainArgs:
    model_name: str = "meta-llama/Llama-2-7b-hf"
    dataset_path: Optional[str] = "./data/glaive_code_full"
    output_dir: str = "./checkpoints/run"
    num_train_epochs: int = 3
    per_device_train_batch_size: int = 1
    gradient_accumulation_steps: int = 1
    learning_rate: float = 2e-4
    lora_r: int = 16
    lora_alpha: Optional[float] = None
    lora_dropout: float = 0.05
    lora_targets: List[str] = field(default_factory=lambda: ["q_proj", "k_proj", "v_proj", "o_proj"])
    max_length: int = 512
    seed: int = 42
    logging_steps: int = 10
    save_strategy: str = "steps"   # steps | epoch | no
    save_steps: int = 100
    save_total_limit: Optional[int] = 3
    gradient_checkpointing: object = False  # True / False / "auto" (memory-aware, see below)
    resume_from_checkpoint: bool = False
    max_steps: int = -1
    warmup_steps: int = 0
    synthetic: bool = False
    synthetic_samples: int = 1024
    synthetic_min_len: Optional[int] = None  # variable-length synthetic rows in [min, max_length]
    pack_sequences: bool = True   # packed varlen rows (no pad compute) when the model supports it
    pack_tokens: int = 0          # >0: micro-batch = whole sequences greedily packed up to this
                                  # many tokens (token-budget batching) instead of a fixed count
    prefetch: int = 2             # batches collated ahead on a host thread (0 = inline)
    init: str = "auto"
    experiment: str = "run"
    strategy: str = ""
    save_final: bool = True
    log_file: Optional[str] = None
    async_save: bool = True
    fuse_accumulation: bool = True  # equal-size accumulation micro-batches as one forward


def model_flops_per_token(cfg, seq_len: int, lora: bool = True) -> float:
    """Approximate training FLOPs/token: fwd 2N + bwd-dX 2N (+ dW 2N when training the base),
    attention 4*L*S*H fwd (x2 for bwd).  Frozen-base LoRA has no weight-gradient GEMMs."""
    n = cfg.num_params() - cfg.vocab_size * cfg.hidden_size  # embedding gather is not a GEMM
    gemm = (4.0 if lora else 6.0) * n
    attn = 4.0 * cfg.num_hidden_layers * seq_len * cfg.hidden_size * 0.5 * 3  # causal, fwd+bwd
    return gemm + attn


class Trainer:
    def __init__(self, args: TrainArgs, ds: DSConfig, env: DistEnv, printer=None):
        self.args, self.ds, self.env = args, ds, env
        self.print = printer or (lambda *a, **k: print(*a, **k, flush=True) if env.is_main else None)
        torch.manual_seed(args.seed)
        if env.device.type == "cuda":
            from ..utils.gemm_tuning import load_tuned_gemms

            load_tuned_gemms()
        dt = ds.torch_dtype
        cfg = get_config(args.model_name)
        self.model_cfg = cfg
        t0 = time.time()
        self.model = build_model(args.model_name, dtype=dt, device=env.device, init=args.init,
                                 seed=args.seed)
        self.print(f"[lumen] model {cfg.name}: {cfg.num_params():,} params, dtype {dt}, "
                   f"built in {time.time() - t0:.1f}s")
        lcfg = LoraConfig(r=args.lora_r, lora_alpha=args.lora_alpha, lora_dropout=args.lora_dropout,
                          target_modules=args.lora_targets)
        apply_lora(self.model, lcfg)
        gc = args.gradient_checkpointing
        gc = gc.lower() if isinstance(gc, str) else gc
        gc = {"true": True, "false": False}.get(gc, gc)
        # True -> the model's default recompute policy (Llama: selective, LUMEN_CKPT_POLICY);
        # "selective" / "full" name one; "auto" is decided after the engine is up (below)
        self.model.gradient_checkpointing = False if gc == "auto" else gc
        self.model.train()
        trainable, total = print_trainable_parameters(self.model, self.print)
        self.n_trainable, self.n_total = trainable, total
        self.engine = ZeroEngine(self.model, ds, env)
        if gc == "auto":
            self.model.gradient_checkpointing = self._auto_checkpointing()
        self.tokenizer = load_tokenizer(args.model_name, cfg.vocab_size)
        pad = getattr(self.tokenizer, "pad_token_id", cfg.eos_token_id)
        self.dataset = build_dataset(args.dataset_path, self.tokenizer, args.max_length,
                                     args.synthetic, args.synthetic_samples, cfg.vocab_size,
                                     seed=args.seed, synthetic_min_len=args.synthetic_min_len)
        self.packed = bool(args.pack_sequences and getattr(self.model, "supports_packing", False))
        if self.packed:
            # token counts rounded to 256 on the GPU: the GEMM M dimension stays on the tuned grid
            self.collator = PackedCollator(pad_id=pad, max_length=args.max_length,
                                           pad_to_multiple_of=256 if env.device.type == "cuda" else 8)
        else:
            self.collator = CausalLMCollator(pad_id=pad, max_length=args.max_length)
        self.sampler = ShardedSampler(len(self.dataset), env.rank, env.world_size, seed=args.seed)
        self.log_history: List[Dict] = []
        self.ckpt = AsyncCheckpointer() if args.async_save else None
        self.flops_per_token = model_flops_per_token(cfg, args.max_length)
        self._plans: Dict[int, List[List[int]]] = {}
        # accumulation groups: fused / run micro-batch by micro-batch / fusable here but not on
        # every rank (vetoed by the cross-rank agreement)
        self.fusion_stats = {"fused": 0, "unfused": 0, "vetoed": 0}

    # ---------------------------------------------------------------------------------------
    def _auto_checkpointing(self):
        """Memory-aware activation checkpointing (``--gradient_checkpointing auto``).

        The reference always recomputes (training/train_baseline.py:181, zero3.py:230) because
        a V100 has 32 GB; full recompute costs ~35% of the step here.  Estimate the activations
        a micro-step keeps for the backward -- ~16 H-wide 16-bit rows per token per layer
        (measured: 14 GB for 8 x 512 Llama-2-7B tokens) -- and pick the cheapest policy whose
        activations fit twice in the HBM left after the model, its shards and optimizer state:
        none, then selective (gate|up output recomputed: ~0.65x the activations, where the model
        has that policy), then full per-layer recompute."""
        env, cfg, a = self.env, self.model_cfg, self.args
        if env.device.type != "cuda":
            return False
        tokens = max(a.pack_tokens, self.ds.micro_batch * a.max_length)
        if a.fuse_accumulation:
            tokens *= self.ds.grad_accum
        from ..parallel.memory_plan import activation_bytes, pick_checkpointing

        est = activation_bytes(cfg, tokens, "none")
        free, _ = torch.cuda.mem_get_info(env.device)
        # blocks the caching allocator holds but no tensor uses are free for activations
        free += torch.cuda.memory_reserved(env.device) - torch.cuda.memory_allocated(env.device)
        # ZeRO-3 allocates at the first micro-steps what is not there yet: the resident
        # gathered units (keep: a whole model copy) with their W^T, and the ring buffers
        co = self.engine.coordinator
        if co is not None:
            free = max(0, free - co.pending_alloc_bytes())
        pols = getattr(type(self.model), "CKPT_POLICIES", None)
        # selective only where every layer's MLP can recompute (frozen, unadapted gate|up/down)
        sel_ok = bool(pols and "selective" in pols
                      and getattr(self.model, "selective_eligible", lambda: False)())
        # per-layer granularity ("selective:N") where the model takes it: recompute only the
        # layers the budget needs
        n_layers = cfg.num_hidden_layers if pols else None
        pick = pick_checkpointing(est, free, sel_ok, n_layers=n_layers)
        if isinstance(pick, str) and pick.split(":")[0] == "full" and not (pols and "full" in pols):
            pick = True
        self.print(f"[lumen] activation checkpointing {pick or 'off'} (auto): "
                   f"~{est / 1e9:.1f} GB of activations per micro-step vs {free / 1e9:.1f} GB "
                   "free HBM (--gradient_checkpointing true|false|selective|full to force)")
        return pick

    @property
    def token_budget(self) -> bool:
        return self.packed and self.args.pack_tokens > 0

    def _length(self, j: int) -> int:
        f = getattr(self.dataset, "length", None)
        n = f(j) if f is not None else len(self.dataset[j]["input_ids"])
        return min(n, self.args.max_length)

    def _plan(self, epoch: int) -> List[List[int]]:
        """This rank's micro-batches (sample indices) for ``epoch``.

        Fixed count: ``micro_batch`` samples each (the tail that does not fill one is dropped,
        like a drop_last loader).  Token budget (``--pack_tokens``): whole sequences in sampler
        order until the next would overflow the budget, tail batch included.  Each rank's shard
        has its own length mix, so the counts differ: every rank truncates to the MIN over ranks
        -- an extra micro-step on one rank would issue ZeRO-3 gathers / reduce-scatters that no
        other rank matches (a hang at the end of the epoch)."""
        if epoch in self._plans:
            return self._plans[epoch]
        idx = self.sampler.indices(epoch)
        if not self.token_budget:
            mb = self.ds.micro_batch
            plan = [idx[i:i + mb] for i in range(0, len(idx) - mb + 1, mb)]
        else:
            budget, plan, cur, n = self.args.pack_tokens, [], [], 0
            for j in idx:
                L = self._length(j)
                if cur and n + L > budget:
                    plan.append(cur)
                    cur, n = [], 0
                cur.append(j)
                n += L
            if cur:
                plan.append(cur)
            if self.env.world_size > 1:
                import torch.distributed as dist

                k = int(all_reduce_scalar(float(len(plan)), op=dist.ReduceOp.MIN))
                plan = plan[:k]
        self._plans = {epoch: plan}
        return plan

    def _batches(self, epoch: int, skip_batches: int):
        for b in self._plan(epoch)[skip_batches:]:
            yield [self.dataset[j] for j in b]

    def _to_device(self, b):
        d = self.env.device
        out = {"input_ids": b["input_ids"].to(d, non_blocking=True),
               "labels": b["labels"].to(d, non_blocking=True),
               "n_valid": b["n_valid"], "n_tokens": b["n_tokens"],
               "micro_steps": b.get("micro_steps", 1)}
        if b.get("cu_seqlens") is not None:
            out["cu_seqlens"] = b["cu_seqlens"]
            out["pos"] = b["pos"].to(d, non_blocking=True)
        return out

    def _batch_stream(self, epoch: int, skip: int):
        """(raw, collated) pairs; collation runs ``prefetch`` batches ahead on a host thread."""
        if self.args.prefetch <= 0:
            return (None, ((raw, self.collator(raw)) for raw in self._batches(epoch, skip)))
        ld = PrefetchLoader(self._batches(epoch, skip), self.collator, depth=self.args.prefetch,
                            pin=self.env.device.type == "cuda")
        return ld, iter(ld)

    def _fused(self, stream):
        """(raw examples, collated batch, micro-steps) per engine forward.  Gradient-accumulation
        fusion: the ``grad_accum`` micro-batches of one optimizer step run as ONE forward /
        backward when they hold the same number of valid labels -- then the fused mean loss is
        exactly the mean of the per-micro-batch means the reference accumulates (HF Trainer
        divides each micro-batch loss by the accumulation steps).  Bigger GEMMs (M = 4096 for
        the ZeRO-3 defaults 2 x 4 x 512 instead of 1024), a quarter of the launches and, under
        ZeRO-3, a quarter of the weight gathers.  Groups start only on an optimizer-step
        boundary; unequal groups run micro-batch by micro-batch."""
        from ..data.collator import fuse_collated

        k = self.ds.grad_accum
        if k <= 1 or not self.args.fuse_accumulation:
            for raw, cb in stream:
                yield raw, cb, 1
            return
        buf = []
        for raw, cb in stream:
            if not buf and self.engine.micro_step % k:
                yield raw, cb, 1          # not at a step boundary (epoch tail): no fusion
                continue
            buf.append((raw, cb))
            if len(buf) < k:
                continue
            local = len({c["n_valid"] for _, c in buf}) == 1
            fuse = local
            if self.env.world_size > 1:
                # one decision for every rank: a fused rank runs ONE forward / backward (one set
                # of ZeRO-3 gathers and bucket reduce-scatters) where an unfused one runs k --
                # mismatched collectives would hang or cross.  Host-side (gloo) agreement: no
                # device sync on the step path
                fuse = agree_all(local)
            self.fusion_stats["fused" if fuse else "vetoed" if local else "unfused"] += 1
            if fuse:
                yield [e for r, _ in buf for e in r], fuse_collated([c for _, c in buf]), k
            else:
                for r, c in buf:
                    yield r, c, 1
            buf = []
        for r, c in buf:
            yield r, c, 1

    def steps_per_epoch(self) -> int:
        if self.token_budget:
            return len(self._plan(0)) // self.ds.grad_accum
        return len(self.sampler) // (self.ds.micro_batch * self.ds.grad_accum)

    def planned_steps(self) -> int:
        """Optimizer steps of the whole run (no ``max_steps``).  Token-budget plans differ in
        length from epoch to epoch (each epoch packs its own permutation), so the total -- which
        sets the HF-linear decay horizon -- sums every epoch's rank-agreed plan; the engine's
        accumulation boundary runs across epochs, hence one floor over the sum."""
        if not self.token_budget:
            return max(self.steps_per_epoch(), 1) * self.args.num_train_epochs
        n = sum(len(self._plan(e)) for e in range(self.args.num_train_epochs))
        return max(n // self.ds.grad_accum, 1)

    def train(self) -> Dict:
        a, ds, env, eng = self.args, self.ds, self.env, self.engine
        start_epoch, skip, skip_b = 0, 0, 0
        if a.resume_from_checkpoint:
            ck = latest_checkpoint(a.output_dir)
            if ck:
                st = load_checkpoint(ck, eng, self.model, env)
                self.log_history = st.get("log_history", [])
                start_epoch = int(st.get("epoch_int", 0))
                skip = int(st.get("samples_in_epoch", 0))
                old_world = int(st.get("world_size", env.world_size))
                if self.token_budget:
                    # token-budget plans are agreed over ranks: the micro-batch count is the
                    # rank-independent position (samples consumed differ per rank)
                    skip_b = int(st.get("batches_in_epoch", 0))
                    if old_world != env.world_size:
                        skip_b = skip_b * old_world // env.world_size
                        self.print("[lumen] warning: --pack_tokens resume at a new world size "
                                   "restarts at the proportional micro-batch (approximate)")
                if old_world != env.world_size:
                    # per-rank position -> same GLOBAL position: step k covers the contiguous
                    # permutation block [k*G, (k+1)*G) at any world size (ShardedSampler)
                    skip = skip * old_world // env.world_size
                    self.print(f"[lumen] resharded checkpoint: world {old_world} -> "
                               f"{env.world_size}")
                if not self.token_budget:
                    skip_b = skip // ds.micro_batch
                self.print(f"[lumen] resumed from {ck} (step {eng.global_step})")
            else:
                self.print("[lumen] no checkpoint found; starting fresh")
        total_steps = a.max_steps if a.max_steps > 0 else self.planned_steps()
        eng.set_total_steps(total_steps)  # HF linear decay (baseline: no DeepSpeed config)
        self.print(f"[lumen] ZeRO-{ds.stage} world={env.world_size} micro={ds.micro_batch} "
                   f"accum={ds.grad_accum} effective batch={ds.train_batch_size} "
                   f"steps={total_steps}")
        prof = StepProfiler(env.rank, self.print)
        # multi-rank: a hung collective ends the job with a diagnosis (exit 19)
        wd = (StepWatchdog.from_env(env.rank, eng.coordinator, "micro-step")
              if env.world_size > 1 else None)
        t_start = time.time()
        tokens = 0
        win_tokens, win_t = 0, t_start
        samples = 0
        loss_acc = torch.zeros((), device=env.device)
        loss_n = 0
        last_loss = float("nan")
        done = eng.global_step >= total_steps
        epoch = start_epoch
        while not done:
            if a.max_steps <= 0 and epoch >= a.num_train_epochs:
                break
            samples_in_epoch = skip
            self._batches_in_epoch = skip_b
            produced = 0
            loader, stream = self._batch_stream(epoch, skip_b)
            for raw, cb, k in self._fused(stream):
                produced += k
                self._batches_in_epoch += k
                if wd is not None:
                    wd.kick()
                b = self._to_device(cb)
                loss = eng.forward(b)
                check_finite("loss", loss, eng.global_step, env.rank)
                eng.backward(loss)
                loss_acc += loss.detach().float() * k  # a fused batch = k micro-step losses
                loss_n += k
                tokens += b["n_tokens"]
                samples += len(raw)
                samples_in_epoch += len(raw)
                if eng.step():
                    prof.step()
                    if ds.dtype != "fp16":  # fp16 overflow is handled by the loss scaler
                        check_finite("grad_norm", eng.last_grad_norm, eng.global_step, env.rank)
                    if eng.global_step % a.logging_steps == 0 or eng.global_step == total_steps:
                        l = all_reduce_scalar(float(loss_acc.item()) / max(loss_n, 1)) / env.world_size
                        gn = float(eng.last_grad_norm.item()) if eng.last_grad_norm is not None else 0.0
                        rec = {"loss": round(l, 4), "grad_norm": gn, "learning_rate": eng.last_lr,
                               "epoch": round(epoch + samples_in_epoch / max(len(self.sampler), 1), 4),
                               "step": eng.global_step}
                        now = time.time()
                        el = now - t_start
                        rec["tokens_per_second"] = round(tokens * env.world_size / max(el, 1e-9), 1)
                        # steady-state rate over the last logging window (non-pad tokens)
                        rec["window_tokens_per_second"] = round(
                            (tokens - win_tokens) * env.world_size / max(now - win_t, 1e-9), 1)
                        win_tokens, win_t = tokens, now
                        self.log_history.append(rec)
                        self.print(json.dumps(rec))
                        if ds.wall_clock_breakdown:
                            br = eng.timers.pop()
                            self.print("[lumen] time (ms) | " + " | ".join(
                                f"{k}: {v * 1e3:.2f}" for k, v in sorted(br.items())))
                        last_loss = l
                        loss_acc.zero_()
                        loss_n = 0
                    if (a.save_strategy == "steps" and a.save_steps > 0
                            and eng.global_step % a.save_steps == 0):
                        self._save(epoch, samples_in_epoch)
                    if self.ckpt is not None and os.environ.get("LUMEN_FAULT_STEP"):
                        self.ckpt.wait()  # injected crashes hit after the last save landed
                    maybe_inject_fault(eng.global_step, env.rank)
                    if eng.global_step >= total_steps:
                        done = True
                        break
            if loader is not None:
                loader.close()
            skip, skip_b = 0, 0
            if produced == 0:
                break
            if not done and a.save_strategy == "epoch":
                self._save(epoch + 1, 0)
            epoch += 1
        prof.close()
        eng.close()  # no ZeRO-3 gather left in flight past the loop
        if wd is not None:
            wd.close()
        if self.ckpt is not None:
            self.ckpt.wait()  # the last periodic checkpoint is complete before we report / exit
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        elapsed = time.time() - t_start
        if loss_n:
            last_loss = all_reduce_scalar(float(loss_acc.item()) / loss_n) / env.world_size
        if a.save_final:
            self.save_final()
        tps = all_reduce_scalar(tokens) / max(elapsed, 1e-9)
        sps = all_reduce_scalar(samples) / max(elapsed, 1e-9)
        peak = (torch.cuda.max_memory_allocated(env.device) / 1e9
                if env.device.type == "cuda" else 0.0)
        return {"training_time_hours": elapsed / 3600.0, "samples_per_second": sps,
                "tokens_per_second": tps, "peak_memory_gb": peak, "final_loss": last_loss,
                "global_step": eng.global_step, "skipped_steps": eng.skipped_steps,
                "tflops_per_gpu": tps * self.flops_per_token / env.world_size / 1e12}

    def _trainer_state(self, epoch: int, samples_in_epoch: int) -> Dict:
        return {"global_step": self.engine.global_step, "epoch_int": epoch,
                "samples_in_epoch": samples_in_epoch,
                "batches_in_epoch": getattr(self, "_batches_in_epoch", 0) if samples_in_epoch else 0,
                "log_history": self.log_history,
                "world_size": self.env.world_size, "zero_stage": self.ds.stage,
                "train_batch_size": self.ds.train_batch_size, "args": asdict(self.args)}

    def _save(self, epoch: int, samples_in_epoch: int):
        save = self.ckpt.save if self.ckpt is not None else save_checkpoint
        p = save(self.args.output_dir, self.engine, self.model,
                 self._trainer_state(epoch, samples_in_epoch), self.env,
                 self.args.save_total_limit, self.args.model_name)
        self.print(f"[lumen] {'saving' if self.ckpt is not None else 'saved'} {p}")

    def save_final(self):
        final = os.path.join(self.args.output_dir, "final")
        if self.env.is_main:
            save_adapter(self.model, final, self.args.model_name)
            self.tokenizer.save_pretrained(final)
        barrier()
        self.print(f"[lumen] final adapter saved to {final}")
