"""Serving engine: continuous batching over the paged-KV model runner.

Replaces the vLLM 0.6 engine the reference declares (README.md:10,16; requirements.txt:17-18):
``LLMEngine`` is the synchronous core (add_request / step / generate), ``AsyncEngine`` runs it
on a background thread and streams tokens to asyncio consumers (the OpenAI API server).
Adapters from training (PEFT dir) are merged into the base weights at load.
With ``tp_size > 1`` rank 0 runs this engine and ranks 1..N-1 run ``worker_loop``.
"""
from __future__ import annotations

import asyncio
import os
import queue
import threading
import time
import uuid
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Union

import numpy as np
import torch
import torch.distributed as dist

from ..models import build_model, get_config
from .block_manager import BlockManager
from .model_runner import ModelRunner, ServeWeights, StepInput, kv_bytes_per_token
from .scheduler import Batch, Scheduler, SchedulerConfig
from .sequence import SamplingParams, Sequence, Status


@dataclass
class EngineConfig:
    model: str = "meta-llama/Llama-2-7b-hf"
    adapter: Optional[str] = None           # PEFT adapter dir to merge (training output)
    dtype: str = "bf16"
    max_model_len: int = 4096
    block_size: int = 16
    gpu_memory_utilization: float = 0.90
    num_blocks: Optional[int] = None
    max_num_seqs: int = 256
    # tokens per engine step (decode rows + prefill chunks): bounds the time a prefill can add
    # to a step, i.e. the inter-token latency of the running streams (chunked prefill)
    max_num_batched_tokens: int = 2048
    # x budget while at most max_num_seqs // 4 sequences decode (scheduler.SchedulerConfig).
    # Off by default: at x2 on the 256-request burst it moved TTFT p50 by -8% / +8% over two
    # runs and ITL p99 by +3-4 ms (profiles/r3d/serve_boost)
    prefill_boost: int = 1
    # "chunked": every step decodes all running streams and fills the rest of the budget with
    # prefill chunks (mixed steps: bounded inter-token latency); "prefill_first": vLLM 0.6.0's
    # default (the version the reference pins) -- prefill-only steps while prompts wait, decode
    # steps otherwise (scheduler.py)
    scheduling_policy: str = "chunked"
    tp_size: int = 1
    seed: int = 0
    use_graphs: bool = True
    device: Optional[str] = None
    init: str = "auto"
    # multi-LoRA serving (vLLM --enable-lora): {served name: PEFT adapter dir}, kept un-merged
    lora_modules: Optional[Dict[str, str]] = None
    max_loras: int = 4
    # async scheduling (TP = 1): step t+1 is scheduled, built and launched while step t runs;
    # its decode tokens come from step t's sampled tokens ON THE DEVICE, and step t's tokens
    # reach the host afterwards (EOS / stop ids are seen one step late: one wasted row)
    async_scheduling: bool = True
    # KV-cache element type: "auto" = model dtype; "fp8" = e4m3 (vLLM --kv-cache-dtype fp8):
    # twice the cache capacity and half the K/V bytes per decode step, at fp8 K/V precision
    kv_cache_dtype: str = "auto"
    # automatic prefix caching (vLLM --enable-prefix-caching): prompts share the cached K/V of
    # equal leading full blocks; finished sequences' blocks stay cached until evicted
    enable_prefix_caching: bool = False
    # speculative decoding by prompt lookup (vLLM --speculative-model "[ngram]"): up to this many
    # draft tokens per greedy sequence, copied from where the sequence's last n tokens (n from
    # ngram_max down to ngram_min) occurred before; a decode step then verifies every draft in
    # one forward (0 = off).  Scheduling is synchronous while it is on.
    num_speculative_tokens: int = 0
    ngram_max: int = 4
    ngram_min: int = 1
    # a verify step is a mixed forward (slower than a graph-replayed decode step): it runs only
    # when at least this fraction of the decode rows has a draft; a sequence whose drafts were
    # all rejected backs off (1, 3, 7 .. 63 steps) before it drafts again
    spec_min_fraction: float = 0.5
    # the prompt-lookup index covers the n-grams of the last ngram_window tokens of a sequence
    # (int keys, pruned as the window slides): at most ngram_window * (ngram_max - ngram_min + 1)
    # dict entries per sequence -- 4 * 1024 with the defaults, ~0.4 MB; 256 sequences ~100 MB
    ngram_window: int = 1024


_DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def apply_penalties(logits: torch.Tensor, seqs: List[Sequence]) -> torch.Tensor:
    """Presence / frequency / repetition penalties on the rows of ``logits`` (f32 result), one
    scatter-add of the rows' token ids into a [rows, V] count table on the device.  Order as in
    vLLM's ``apply_penalties``: the repetition penalty first (on the raw logit's sign), then the
    frequency and presence subtractions."""
    out = logits.float().clone()
    rows = [i for i, s in enumerate(seqs) if s.params.has_penalties]
    V = out.shape[1]
    dev = out.device

    def counts(id_lists):
        L = max((len(x) for x in id_lists), default=0)
        c = torch.zeros(len(id_lists), V + 1, dtype=torch.float32, device=dev)
        if L:
            ids = torch.full((len(id_lists), L), V, dtype=torch.long)
            for j, x in enumerate(id_lists):
                if x:
                    ids[j, :len(x)] = torch.tensor(x, dtype=torch.long)
            ids = ids.to(dev)
            c.scatter_add_(1, ids, torch.ones_like(ids, dtype=torch.float32))
        return c[:, :V]

    sel = [seqs[i] for i in rows]
    ridx = torch.tensor(rows, dtype=torch.long, device=dev)
    lg = out[ridx]
    rp = torch.tensor([s.params.repetition_penalty for s in sel], device=dev)[:, None]
    if bool((rp != 1.0).any()):
        seen = (counts([s.all_ids for s in sel]) > 0) & (rp != 1.0)
        lg = torch.where(seen, torch.where(lg > 0, lg / rp, lg * rp), lg)
    out_c = counts([s.output_ids for s in sel])
    fp = torch.tensor([s.params.frequency_penalty for s in sel], device=dev)[:, None]
    pp = torch.tensor([s.params.presence_penalty for s in sel], device=dev)[:, None]
    lg = lg - (fp * out_c + pp * (out_c > 0).float())
    out[ridx] = lg
    return out


class LLMEngine:
    def __init__(self, cfg: EngineConfig, model=None, tokenizer=None):
        self.cfg = cfg
        self.tp = cfg.tp_size
        self.rank = dist.get_rank() if (self.tp > 1 and dist.is_initialized()) else 0
        if cfg.device:
            dev = torch.device(cfg.device)
        elif torch.cuda.is_available():
            dev = torch.device("cuda", torch.cuda.current_device())
        else:
            dev = torch.device("cpu")
        self.device = dev
        if dev.type == "cuda":
            from ..utils.gemm_tuning import load_tuned_gemms

            load_tuned_gemms()  # tuned hipBLASLt algorithms for the prefill/decode GEMM shapes
        dt = _DT[cfg.dtype] if dev.type == "cuda" else torch.float32
        if model is None:
            model = build_model(cfg.model, dtype=dt, device=dev, init=cfg.init, seed=cfg.seed)
        if cfg.adapter:
            from ..lora import load_adapter, merge_lora

            load_adapter(model, cfg.adapter)
            merge_lora(model)
        model.eval()
        self.model_config = model.config
        tp_group = dist.group.WORLD if self.tp > 1 else None
        if self.tp > 1:
            # the host side of the step broadcast (lumen/serve/tp.py): created collectively here,
            # where every rank constructs its engine
            from ..parallel.dist import host_group

            host_group()
        self.weights = ServeWeights(model, self.rank, self.tp)
        if cfg.kv_cache_dtype not in ("auto", "fp8"):
            raise ValueError(f"kv_cache_dtype must be 'auto' or 'fp8', got {cfg.kv_cache_dtype}")
        self.kv_dtype = torch.float8_e4m3fn if cfg.kv_cache_dtype == "fp8" else dt
        nb = cfg.num_blocks or self._auto_blocks(self.kv_dtype)
        if self.tp > 1 and dist.is_initialized():
            # one block count for the whole TP group: rank 0 schedules block ids that every
            # worker's cache must hold (free memory, hence the auto count, can differ per rank)
            from ..parallel.dist import host_group

            t = torch.tensor([nb], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=host_group())
            nb = int(t.item())
        self.blocks = BlockManager(nb, cfg.block_size, prefix_caching=cfg.enable_prefix_caching)
        car = None
        if self.tp > 1 and dev.type == "cuda":
            # TP decode: row-parallel sums on the custom IPC all-reduce, which also lets the
            # decode buckets be captured in hipGraphs (collective: every rank builds it here)
            from ..parallel.custom_ar import maybe_custom_allreduce

            esz = torch.empty((), dtype=dt).element_size()
            rows = min(256, cfg.max_num_seqs)
            vshard = model.config.vocab_size // self.tp
            car = maybe_custom_allreduce(
                tp_group, dev, max(8 << 20, rows * model.config.hidden_size * esz,
                                   rows * vshard * esz))
        self.runner = ModelRunner(self.weights, nb, cfg.block_size, dev, cfg.max_model_len,
                                  tp_group, use_graphs=cfg.use_graphs,
                                  max_graph_batch=min(256, cfg.max_num_seqs), custom_ar=car,
                                  kv_dtype=self.kv_dtype)
        self.lora_names: List[str] = []
        if cfg.lora_modules:
            from .multi_lora import MultiLoRA

            self.runner.lora = MultiLoRA(model.config, cfg.lora_modules, cfg.max_loras, self.rank,
                                         self.tp, dev, dt)
            self.lora_names = list(self.runner.lora.names)
        self._pinned: List[Optional[torch.Tensor]] = [None, None]
        self._pinned_ready: List[Optional[object]] = [None, None]
        self._pin_i = 0
        # TP > 1 too: a step is broadcast when it is launched, its decode tokens straight from
        # the device (gathered from the previous step's samples), so workers never wait for
        # rank 0's host to see the tokens
        self.spec_k = max(0, int(cfg.num_speculative_tokens))
        # drafting reads every sequence's latest token on the host: no step in flight
        self.async_sched = bool(cfg.async_scheduling) and self.spec_k == 0
        self._inflight: Optional[dict] = None
        self.scheduler = Scheduler(SchedulerConfig(
            cfg.max_num_seqs, cfg.max_num_batched_tokens, cfg.max_model_len,
            prefill_boost=max(1, int(cfg.prefill_boost)), policy=cfg.scheduling_policy),
            self.blocks)
        if tokenizer is None:
            from ..data.tokenizer import load_tokenizer

            tokenizer = load_tokenizer(cfg.model, self.model_config.vocab_size)
        self.tokenizer = tokenizer
        self.eos_id = getattr(tokenizer, "eos_token_id", self.model_config.eos_token_id)
        self.step_count = 0
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "steps": 0, "requests": 0,
                      "finished": 0, "overlapped_steps": 0, "spec_proposed": 0,
                      "spec_accepted": 0, "spec_steps": 0}

    # --------------------------------------------------------------------------------------
    def _auto_blocks(self, dt) -> int:
        per_tok = kv_bytes_per_token(self.model_config, torch.tensor([], dtype=dt).element_size(),
                                     self.tp)
        per_block = per_tok * self.cfg.block_size
        if self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            budget = free - (1 - self.cfg.gpu_memory_utilization) * total
            budget -= 4 << 30  # activations / graphs / workspace headroom
            if os.environ.get("LUMEN_SHARED_GPU_REHEARSAL") == "1" and self.tp > 1:
                # ranks sharing one device (rehearsal) each see the same free memory before any
                # of them allocates: split it, or the last rank to allocate runs out
                budget /= self.tp
        else:
            budget = 256 << 20
        nb = int(max(budget, per_block * 64) // per_block)
        cap = self.cfg.max_num_seqs * ((self.cfg.max_model_len + self.cfg.block_size - 1)
                                       // self.cfg.block_size) + 64
        return max(64, min(nb, cap))

    def encode(self, prompt: Union[str, List[int]]) -> List[int]:
        if isinstance(prompt, str):
            return self.tokenizer.encode(prompt)
        return list(prompt)

    def add_request(self, prompt: Union[str, List[int]], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None, lora: Optional[str] = None) -> Sequence:
        params = params or SamplingParams()
        ids = self.encode(prompt)
        if not ids:
            raise ValueError("empty prompt")
        budget = self.cfg.max_model_len - len(ids)
        if budget < 1:
            raise ValueError(f"prompt ({len(ids)} tokens) does not fit max_model_len "
                             f"{self.cfg.max_model_len}")
        if params.max_tokens > budget:
            params.max_tokens = budget
        if params.prompt_logprobs is not None and self.tp > 1:
            raise ValueError("prompt_logprobs is served at tensor-parallel size 1 only")
        seq = Sequence(ids, params, request_id or uuid.uuid4().hex)
        if lora:
            if self.runner.lora is None or lora not in self.lora_names:
                raise ValueError(f"unknown LoRA adapter '{lora}' (serving: {self.lora_names})")
            seq.lora_slot = self.runner.lora.slot_of(lora)
        self.scheduler.add(seq)
        self.stats["requests"] += 1
        return seq

    def abort(self, request_id: str) -> None:
        self.scheduler.abort(request_id)

    @property
    def has_work(self) -> bool:
        return self.scheduler.has_work or self._inflight is not None

    # --------------------------------------------------------------------------------------
    def _build_input(self, batch: Batch) -> StepInput:
        """Host-side step metadata, vectorised with numpy and shipped in ONE host-to-device copy
        (a Python/torch loop per sequence cost ~10 ms per 256-sequence decode step, a third of
        the step).  Rows: prefill chunks first, then decode tokens."""
        bm = self.blocks
        bs = bm.block_size
        use_lora = self.runner.lora is not None
        toks, pos, slots, lora = [], [], [], []
        cu, kv_lens, ptables = [0], [], []
        for s, c in batch.prefills:
            a = s.num_cached
            ids = s.all_ids + s.draft if s.draft else s.all_ids
            toks.append(np.asarray(ids[a:a + c], dtype=np.int64))
            p = np.arange(a, a + c, dtype=np.int64)
            pos.append(p)
            tbl = np.asarray(bm.tables[s.seq_id], dtype=np.int64)
            slots.append(tbl[p // bs] * bs + p % bs)
            cu.append(cu[-1] + c)
            kv_lens.append(a + c)
            ptables.append(tbl)
            if use_lora:
                lora.append(np.full(c, s.lora_slot, dtype=np.int64))
        # prompt_logprobs: the row at position p scores prompt token p + 1
        prows: List[int] = []
        pmeta = []
        for i, (s, c) in enumerate(batch.prefills):
            if s.params.prompt_logprobs is None:
                continue
            a = s.num_cached
            hi = min(a + c, len(s.prompt_ids) - 1)
            if hi > a:
                pmeta.append((s, a + 1, hi - a, len(prows)))
                prows.extend(range(cu[i], cu[i] + hi - a))
        Tp = cu[-1]
        N = len(batch.decodes)
        parts = toks + pos + slots
        dec_bt = None
        maxb_d = 0
        if N:
            tables = [bm.tables[s.seq_id] for s in batch.decodes]
            lens = np.fromiter((s.length for s in batch.decodes), dtype=np.int64, count=N)
            dtok = np.fromiter((s.last_token for s in batch.decodes), dtype=np.int64, count=N)
            maxb_d = max(len(t) for t in tables)
            dec_bt = np.zeros((N, maxb_d), dtype=np.int64)
            for i, t in enumerate(tables):
                dec_bt[i, :len(t)] = t
            dpos = lens - 1
            dslots = dec_bt[np.arange(N), dpos // bs] * bs + dpos % bs
            # decode rows go after the prefill rows in each of tokens / positions / slots
            parts = toks + [dtok] + pos + [dpos] + slots + [dslots]
            if use_lora:
                lora.append(np.fromiter((s.lora_slot for s in batch.decodes), dtype=np.int64,
                                        count=N))
        T = Tp + N
        P = len(batch.prefills)
        maxb_p = max((len(t) for t in ptables), default=0)
        extra = []
        if P:
            pt = np.zeros((P, maxb_p), dtype=np.int64)
            for i, t in enumerate(ptables):
                pt[i, :len(t)] = t
            extra += [pt.reshape(-1), np.asarray(kv_lens, dtype=np.int64)]
        if N:
            extra += [dec_bt.reshape(-1), lens]
        src = None
        if N and self._inflight is not None:
            # decode inputs still being sampled by the in-flight step: row of its token tensor
            row = self._inflight["row"]
            src = np.fromiter((row.get(s.seq_id, -1) if s.has_pending else -1
                               for s in batch.decodes), dtype=np.int64, count=N)
            if not (src >= 0).any():
                src = None
            else:
                extra.append(src)
        if batch.kind == "verify":
            # speculative verification: every row of a drafted chunk is scored
            done_rows = list(range(Tp))
            ps = [s.params for s, c in batch.prefills for _ in range(c)]
            ps += [s.params for s in batch.decodes]
        else:
            n_done = len(batch.completing())
            done_rows = [cu[i + 1] - 1 for i, (s, c) in enumerate(batch.prefills)
                         if s.num_cached + c == s.length]
            assert len(done_rows) == n_done
            ps = [s.params for s in batch.sampled]
        rows = np.concatenate([np.asarray(done_rows, dtype=np.int64),
                               np.arange(Tp, T, dtype=np.int64)])
        extra.append(rows)
        R = len(rows)
        if R:
            # sampling parameters of the sampled rows ride in the same async copy: building them
            # with torch.tensor(list, device=...) is a blocking copy -- a stream synchronise per
            # step that would serialise the host with the GPU and undo async scheduling
            extra += [np.fromiter((p.temperature for p in ps), np.float64, R).view(np.int64),
                      np.fromiter((p.top_p for p in ps), np.float64, R).view(np.int64),
                      np.fromiter((p.top_k for p in ps), np.int64, R)]
        if prows:
            extra.append(np.asarray(prows, dtype=np.int64))
        if use_lora:
            extra.append(np.concatenate(lora))
        host = np.concatenate([np.concatenate(parts)] + extra)
        dev = self._to_device(host)
        o = 3 * T
        inp = StepInput("mixed" if batch.kind == "verify" else batch.kind, dev[:T],
                        dev[T:2 * T].int(), dev[2 * T:3 * T], cu)
        if P:
            inp.prefill_tables = dev[o:o + P * maxb_p].view(P, maxb_p).int()
            o += P * maxb_p
            inp.kv_lens = kv_lens
            inp.kv_lens_t = dev[o:o + P].int()
            o += P
        if N:
            inp.block_tables = dev[o:o + N * maxb_d].view(N, maxb_d).int()
            o += N * maxb_d
            inp.context_lens = dev[o:o + N].int()
            o += N
            inp.max_context = int(lens.max())
        if src is not None:
            # dependent decode tokens: gathered from the previous step's sampled tokens here,
            # on the stream, before the step reads (or its graph copies in) its token row
            s_dev = dev[o:o + N]
            o += N
            prev = self._inflight["toks"]
            inp.tokens[Tp:] = torch.where(s_dev >= 0, prev[s_dev.clamp(min=0)], inp.tokens[Tp:])
        inp.sample_rows = dev[o:o + R]
        o += R
        if R:
            inp.temps = dev[o:o + R].view(torch.float64).float()
            inp.top_ps = dev[o + R:o + 2 * R].view(torch.float64).float()
            inp.top_ks = dev[o + 2 * R:o + 3 * R].int()
            o += 3 * R
        if prows:
            inp.extra_rows = dev[o:o + len(prows)]
            inp.prompt_meta = pmeta
            o += len(prows)
        if use_lora:
            inp.lora_ids = dev[o:o + T].int()
        return inp

    def _to_device(self, host: "np.ndarray") -> torch.Tensor:
        t = torch.from_numpy(host)
        if self.device.type != "cuda":
            return t
        # two pinned staging buffers, alternating: the copy of step t-1 (queued behind step t-2's
        # kernels) never makes the host wait while it builds step t
        i = self._pin_i
        self._pin_i ^= 1
        if self._pinned_ready[i] is not None:
            self._pinned_ready[i].synchronize()  # that buffer's last copy has been read
        if self._pinned[i] is None or self._pinned[i].numel() < t.numel():
            self._pinned[i] = torch.empty(max(t.numel(), 1 << 16), dtype=torch.long).pin_memory()
        buf = self._pinned[i][:t.numel()]
        buf.copy_(t)
        out = buf.to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pinned_ready[i] = ev
        return out

    def _broadcast(self, inp: Optional[StepInput]):
        """TP: ship the step to worker ranks as two int64 tensors (header + payload)."""
        from .tp import pack_step

        pack_step(inp, self.device)

    def step(self) -> List[Sequence]:
        """Run one engine iteration; returns sequences that received a token this step."""
        if not self.async_sched:
            batch = self.scheduler.schedule()
            if batch is None:
                return []
            if self.spec_k and batch.kind == "decode" and self._propose(batch):
                return self._run_verify(batch)
            return self._run_batch(batch)
        batch = self.scheduler.schedule()
        if batch is None:
            return self._resolve()
        if any(s.params.wants_extras for s in batch.seqs):
            # logprob alternatives / prompt scores: this step runs resolved (synchronously)
            done = self._resolve() if self._inflight is not None else []
            batch = self._drop_finished(batch)
            return done + (self._run_batch(batch) if batch is not None else [])
        if self._inflight is not None and self._needs_host_tokens(batch):
            done = self._resolve()     # this step reads real token values on the host
            # the resolved tokens may have finished (EOS / stop id / max_tokens) sequences of
            # the batch just built: their KV tables are freed, so they must not run again
            batch = self._drop_finished(batch)
            if batch is not None:
                self._launch(batch)
            return done
        prev = self._inflight
        self._launch(batch)            # step t+1 is queued behind step t ...
        if prev is None:               # (nothing older in flight: t+1 stays in flight)
            return []
        self.stats["overlapped_steps"] += 1
        return self._resolve(prev)     # ... while the host collects step t's tokens

    @staticmethod
    def _drop_finished(batch: Batch) -> Optional[Batch]:
        """The batch without the sequences that finished after it was scheduled (None if
        nothing is left).  A finished prefill's chunk and a finished decode's row just vanish:
        their blocks were already returned by ``finish_seqs``."""
        pre = [(s, c) for s, c in batch.prefills if not s.finished]
        dec = [s for s in batch.decodes if not s.finished]
        if not pre and not dec:
            return None
        return Batch("mixed" if pre else "decode", pre, dec)

    @staticmethod
    def _needs_host_tokens(batch: Batch) -> bool:
        """Prefill rows re-reading generated tokens (preemption recompute) and penalties need
        the in-flight step's token VALUES on the host."""
        return (any(s.has_pending for s, _ in batch.prefills)
                or any(s.params.has_penalties for s in batch.sampled))

    def _launch(self, batch: Batch) -> None:
        inp = self._build_input(batch)
        if self.tp > 1:
            self._broadcast(inp)
        sampled = batch.sampled
        if batch.kind == "decode":
            logits = self.runner.decode(inp)
        else:
            logits = self.runner.execute(inp)
        self.stats["prefill_tokens"] += inp.num_prefill_rows
        self.stats["decode_tokens"] += len(batch.decodes)
        rec = {"sampled": [], "row": {}, "toks": None}
        if sampled:
            ps = [s.params for s in sampled]
            seed = self.cfg.seed if ps[0].seed is None else ps[0].seed
            if any(p.has_penalties for p in ps):
                logits = apply_penalties(logits, sampled)
            t, lp = self.runner.sample(logits, inp.temps, inp.top_ps, inp.top_ks, seed,
                                       self.step_count, want_logprobs=True)
            R = t.shape[0]
            th = torch.empty(R, dtype=torch.long, pin_memory=self.device.type == "cuda")
            th.copy_(t, non_blocking=True)
            lh = None
            if lp is not None:
                lh = torch.empty(R, dtype=torch.float32, pin_memory=self.device.type == "cuda")
                lh.copy_(lp, non_blocking=True)
            ev = torch.cuda.Event() if self.device.type == "cuda" else None
            if ev is not None:
                ev.record()
            rec.update(toks=t, th=th, lh=lh, ev=ev, sampled=sampled)
        self.scheduler.launched(batch)
        for s, c in batch.prefills:
            s.num_cached += c
        for s in batch.decodes:
            s.num_cached = s.length
        for i, s in enumerate(sampled):
            s.prefilled = True
            rec["row"][s.seq_id] = i
            s.reserve()
        self.stats["steps"] += 1
        self.step_count += 1
        self._inflight = rec if sampled else None

    def _resolve(self, rec: Optional[dict] = None) -> List[Sequence]:
        """Bring a launched step's sampled tokens to the host and apply them."""
        if rec is None:
            rec, self._inflight = self._inflight, None
        if rec is None or not rec["sampled"]:
            return []
        if rec["ev"] is not None:
            rec["ev"].synchronize()
        toks = rec["th"].tolist()
        lps = rec["lh"].tolist() if rec["lh"] is not None else [None] * len(toks)
        nxt = self._inflight if self._inflight is not rec else None
        out, ended = [], []
        for s in rec["sampled"]:
            i = rec["row"].get(s.seq_id)
            if i is None:
                continue
            if s.finished:            # aborted while in flight
                s.n_pending = 0
                continue
            s.fill(int(toks[i]), lps[i], self.eos_id)
            if s.finished:
                ended.append(s)
                if nxt is not None and nxt["row"].pop(s.seq_id, None) is not None:
                    # EOS / stop id seen one step late: the next step's row for it is wasted
                    s.n_pending -= 1
            out.append(s)
        self.runner.check_collectives()
        self.stats["finished"] += len(self.scheduler.finish_seqs(ended))
        return out

    def _run_batch(self, batch: Batch) -> List[Sequence]:
        inp = self._build_input(batch)
        if self.tp > 1:
            self._broadcast(inp)
        sampled = batch.sampled   # before the cache bookkeeping below changes num_cached
        if batch.kind == "decode":
            logits = self.runner.decode(inp)
        else:
            logits = self.runner.execute(inp)
        self.stats["prefill_tokens"] += inp.num_prefill_rows
        self.stats["decode_tokens"] += len(batch.decodes)
        toks, lps = [], []
        if sampled:
            ps = [s.params for s in sampled]
            seed = self.cfg.seed if ps[0].seed is None else ps[0].seed
            if any(p.has_penalties for p in ps):
                logits = apply_penalties(logits, sampled)
            t, lp = self.runner.sample(logits, inp.temps, inp.top_ps, inp.top_ks, seed,
                                       self.step_count, want_logprobs=True)
            toks = t.tolist()
            lps = lp.tolist() if lp is not None else [None] * len(toks)
        tops = self._extras(inp, logits, sampled)
        self.runner.check_collectives()  # a timed-out TP reduction never returns its tokens
        self.scheduler.launched(batch)
        for s, c in batch.prefills:
            s.num_cached += c
        for s in batch.decodes:
            s.num_cached = s.length
        for s, t, lp, top in zip(sampled, toks, lps, tops):
            s.prefilled = True
            s.append(int(t), lp, self.eos_id, top)
        done = self.scheduler.finish(batch)
        self.stats["finished"] += len(done)
        self.stats["steps"] += 1
        self.step_count += 1
        return sampled

    # ---- speculative decoding (prompt lookup) ----------------------------------------------
    @staticmethod
    def _ngram_key(ids: List[int], a: int, b: int) -> int:
        return hash(tuple(ids[a:b]))

    def _lookup(self, ids: List[int], k: int, s: Optional[Sequence] = None) -> List[int]:
        """Up to k tokens that followed the most recent earlier occurrence of the sequence's
        last n tokens (n = ngram_max .. ngram_min) within its last ``ngram_window`` tokens.
        The n-gram index of ``s`` (int hash of the n-gram -> position after it) is extended
        incrementally -- a few dict updates per new token, where a scan of the history cost
        ~60 us per sequence, 15 ms per 256-row step -- and pruned as the window slides, so its
        size is bounded.  A hash collision can only propose a wrong draft, which the verify
        step rejects (outputs stay identical to plain decoding)."""
        lo, hi = max(1, self.cfg.ngram_min), self.cfg.ngram_max
        W = max(1, int(self.cfg.ngram_window))
        idx = s.ngram_idx if s is not None else {}
        upto = s.ngram_upto if s is not None else 0
        L = len(ids)
        start = max(upto, L - 1 - W)
        key = self._ngram_key
        for p in range(start, L - 1):          # n-grams ending before the current suffix
            for n in range(lo, min(hi, p + 1) + 1):
                idx[key(ids, p - n + 1, p + 1)] = p + 1
        if s is not None:
            # n-grams ending before the window start leave the index (unless a later
            # occurrence has taken the key over)
            for p in range(max(0, upto - W - 1), max(0, L - 1 - W)):
                for n in range(lo, min(hi, p + 1) + 1):
                    kk = key(ids, p - n + 1, p + 1)
                    if idx.get(kk) == p + 1:
                        del idx[kk]
            s.ngram_upto = max(upto, L - 1)
        for n in range(min(hi, L - 1), lo - 1, -1):
            j = idx.get(key(ids, L - n, L))
            if j is not None and j < L:
                return ids[j:j + k]
        return []

    def _propose(self, batch: Batch) -> bool:
        """Drafts for the greedy decode rows of ``batch`` (``Sequence.draft``), their KV slots
        reserved; False when nothing was drafted.  The spec_min_fraction check and the token
        budget (verify rows + plain decode rows <= max_num_batched_tokens) are applied BEFORE
        any block is reserved, so dropped drafts never grow a table or evict cached blocks."""
        if any(s.params.wants_extras for s in batch.decodes):
            return False                      # alternatives are computed on the plain path
        cand = []
        for s in batch.decodes:
            p = s.params
            if p.temperature > 0 or p.has_penalties or p.wants_extras:
                continue
            if s.spec_wait > 0:
                s.spec_wait -= 1
                continue
            room = min(self.spec_k, p.max_tokens - len(s.output_ids) - 1,
                       self.cfg.max_model_len - s.length - 1)
            if room <= 0:
                continue
            d = self._lookup(s.all_ids, room, s)
            if d:
                cand.append((s, d))
        # budget: every decode row costs 1, a draft adds len(d) verify rows
        spare = self.cfg.max_num_batched_tokens - len(batch.decodes)
        kept = []
        for s, d in cand:
            d = d[:max(0, spare)]
            if not d:
                break
            spare -= len(d)
            kept.append((s, d))
        if not kept or len(kept) < self.cfg.spec_min_fraction * len(batch.decodes):
            for s, _ in cand:             # too few drafts to pay for a verify step
                s.spec_wait = 3           # (and look again in a few steps, not every step)
            return False
        drafted = []
        for s, d in kept:
            need = s.length + len(d) + 1
            extra = self.blocks.blocks_needed(need) - len(self.blocks.tables.get(s.seq_id, []))
            if extra > self.blocks.num_free:
                continue                      # no blocks for the draft: plain decode row
            self.blocks.ensure(s.seq_id, need)
            s.draft = d
            drafted.append(s)
        return bool(drafted)

    def _run_verify(self, batch: Batch) -> List[Sequence]:
        """One forward over [last token + draft] chunks of the drafted sequences and the other
        decode rows: the longest draft prefix the model's argmax agrees with is accepted, plus
        the model's own next token -- greedy outputs identical to one-token decoding."""
        drafted = [s for s in batch.decodes if s.draft]
        vb = Batch("verify", [(s, 1 + len(s.draft)) for s in drafted],
                   [s for s in batch.decodes if not s.draft])
        inp = self._build_input(vb)
        if self.tp > 1:
            self._broadcast(inp)
        logits = self.runner.execute(inp)
        # drafted rows are greedy (argmax); the undrafted decode rows keep their own sampling
        if any(s.params.has_penalties for s in vb.decodes):
            logits = apply_penalties(logits, [s for s, c in vb.prefills for _ in range(c)]
                                     + vb.decodes)
        p0 = vb.seqs[0].params
        t, lp = self.runner.sample(logits, inp.temps, inp.top_ps, inp.top_ks,
                                   self.cfg.seed if p0.seed is None else p0.seed,
                                   self.step_count, want_logprobs=True)
        amv = t.tolist()
        lpv = lp.tolist() if lp is not None else [None] * len(amv)
        self.runner.check_collectives()
        self.stats["prefill_tokens"] += inp.num_prefill_rows
        self.stats["decode_tokens"] += len(vb.decodes)
        self.stats["spec_steps"] += 1
        r = 0
        out = []
        for s, c in vb.prefills:
            d, s.draft = s.draft, []
            acc = 0
            while acc < len(d) and amv[r + acc] == d[acc]:
                acc += 1
            self.stats["spec_proposed"] += len(d)
            self.stats["spec_accepted"] += acc
            if acc:
                s.spec_misses = 0
            else:
                s.spec_misses += 1
                s.spec_wait = min(2 ** s.spec_misses - 1, 63)
            for t, lp in zip(d[:acc] + [amv[r + acc]], lpv[r:r + acc + 1]):
                s.append(int(t), lp, self.eos_id)
                if s.finished:
                    break
            s.num_cached = s.length - 1       # K/V valid up to the last accepted input
            r += c
            out.append(s)
        for s in vb.decodes:
            s.num_cached = s.length
            s.append(int(amv[r]), lpv[r], self.eos_id)
            r += 1
            out.append(s)
        self.stats["finished"] += len(self.scheduler.finish(vb))
        self.stats["steps"] += 1
        self.step_count += 1
        return out

    def _extras(self, inp: StepInput, logits: torch.Tensor, sampled: List[Sequence]) -> list:
        """Host lists of the ``top_logprobs`` alternatives of each sampled row (None where not
        asked; from the distribution the row was sampled from: logits / temperature, raw when
        greedy), and the prompt scores of this step's prefill rows (stored on the sequences)."""
        tops: list = [None] * len(sampled)
        ks = [s.params.top_logprobs for s in sampled]
        if any(ks):
            z = logits.float()
            t = inp.temps.float()[:, None]
            z = torch.where(t > 0, z / t.clamp(min=1e-6), z)
            v, ix = torch.log_softmax(z, -1).topk(max(ks), -1)
            v, ix = v.tolist(), ix.tolist()
            tops = [list(zip(ix[i][:k], v[i][:k])) if k else None for i, k in enumerate(ks)]
        meta = inp.prompt_meta
        if meta:
            lp = torch.log_softmax(self.runner.extra_logits.float(), -1)
            tgt = torch.tensor([t for s, j0, n, _ in meta for t in s.prompt_ids[j0:j0 + n]],
                               dtype=torch.long, device=lp.device)
            tl = lp.gather(1, tgt[:, None])[:, 0].tolist()
            kp = max(s.params.prompt_logprobs for s, *_ in meta)
            pv = pi = None
            if kp:
                pv, pi = lp.topk(kp, -1)
                pv, pi = pv.tolist(), pi.tolist()
            for s, j0, n, r0 in meta:
                if not s.prompt_scores:
                    s.prompt_scores.append(None)   # the first token has no prefix to score it
                k = s.params.prompt_logprobs
                for q in range(n):
                    if j0 + q != len(s.prompt_scores):
                        continue                   # scored before (recompute after preemption)
                    alts = list(zip(pi[r0 + q][:k], pv[r0 + q][:k])) if k else []
                    s.prompt_scores.append((tl[r0 + q], alts))
        return tops

    def generate(self, prompts: Iterable[Union[str, List[int]]],
                 params: Optional[SamplingParams] = None) -> List[Sequence]:
        seqs = [self.add_request(p, SamplingParams(**vars(params)) if params else None)
                for p in prompts]
        while any(not s.finished for s in seqs):
            self.step()
        return seqs

    def shutdown(self):
        if self.tp > 1:
            self._broadcast(None)


class AsyncEngine:
    """Background-thread engine loop + asyncio streaming (OpenAI server backend)."""

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self._inbox: "queue.Queue" = queue.Queue()
        self._streams: Dict[str, tuple] = {}
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="lumen-engine", daemon=True)
        self._thread.start()

    def _loop(self):
        eng = self.engine
        while not self._stop.is_set():
            try:
                while True:
                    op = self._inbox.get_nowait()
                    if op[0] == "add":
                        _, prompt, params, rid, lora = op
                        try:
                            seq = eng.add_request(prompt, params, rid, lora)
                            self._push(rid, ("start", seq))
                        except Exception as e:  # bad request -> report to its stream
                            self._push(rid, ("error", str(e)))
                    elif op[0] == "abort":
                        eng.abort(op[1])
            except queue.Empty:
                pass
            if not eng.has_work:
                time.sleep(0.0005)
                continue
            try:
                seqs = eng.step()
            except Exception as e:  # surface engine failures to every open stream
                for rid in list(self._streams):
                    self._push(rid, ("error", repr(e)))
                raise
            for s in seqs:
                self._push(s.request_id, ("token", s))

    # -- interface shared with frontend.EngineCoreClient (what the API server reads) ---------
    @property
    def tokenizer(self):
        return self.engine.tokenizer

    @property
    def model_name(self) -> str:
        return self.engine.cfg.model

    @property
    def max_model_len(self) -> int:
        return self.engine.cfg.max_model_len

    @property
    def eos_id(self):
        return self.engine.eos_id

    def live_stats(self) -> dict:
        sch = self.engine.scheduler
        return {"kv_usage": self.engine.blocks.usage(), "running": len(sch.running),
                "waiting": len(sch.waiting), "preemptions": sch.num_preemptions,
                "prefix_hit_rate": self.engine.blocks.hit_rate}

    def _push(self, rid, item):
        st = self._streams.get(rid)
        if st is None:
            return
        loop, q = st
        loop.call_soon_threadsafe(q.put_nowait, item)

    @property
    def lora_names(self) -> List[str]:
        return list(self.engine.lora_names)

    async def stream(self, prompt, params: SamplingParams, request_id: Optional[str] = None,
                     lora: Optional[str] = None):
        """Async generator of (sequence, new_token_count) updates until finished."""
        rid = request_id or uuid.uuid4().hex
        q: asyncio.Queue = asyncio.Queue()
        self._streams[rid] = (asyncio.get_running_loop(), q)
        self._inbox.put(("add", prompt, params, rid, lora))
        kind, payload = "start", None
        try:
            while True:
                kind, payload = await q.get()
                if kind == "error":
                    raise ValueError(payload)
                if kind == "start":
                    continue
                yield payload
                if payload.finished:
                    break
        finally:
            self._streams.pop(rid, None)
            if not (kind == "token" and payload is not None and payload.finished):
                self._inbox.put(("abort", rid))  # client went away: free its KV blocks

    def shutdown(self):
        self._stop.set()
        self._thread.join(timeout=5)
