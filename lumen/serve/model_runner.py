"""Serving model runner: paged-KV mixed prefill / decode of Llama-family models on MI355X.

Per layer (token-major activations, no autograd):
    fused add+RMSNorm (HIP) -> q|k|v GEMM (hipBLASLt) -> RoPE on q,k at each token's position +
    K/V scattered into the paged cache by slot (one HIP kernel) -> attention
    [prefill chunks: 32x32x16 flash forward over the paged cache, queries offset by the cached
    context (whole prompts, chunks of long prompts); decode rows: HIP paged decode]
    -> o GEMM (+ all-reduce under TP) -> fused add+RMSNorm -> gate|up GEMM -> SwiGLU (HIP)
    -> down GEMM (+ all-reduce) ; final norm on the sampled rows only -> LM head -> HIP sampler.
A "mixed" step packs [prefill chunk tokens | decode tokens] into one forward (every GEMM sees
all of them); a pure decode step replays a hipGraph.

Tensor parallelism: Megatron-style column split of q|k|v and gate|up by
heads / FFN columns, row split of o and down followed by an all-reduce over the TP group.
Rank 0 owns the scheduler; every step it broadcasts one int64 metadata tensor (token ids,
positions, slots, block tables, lengths) so worker ranks run the same kernels (no pickling).
Decode steps are captured in HIP graphs per batch-size bucket (static input buffers), which
removes the per-kernel launch cost that otherwise dominates small-batch decode.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence as Seq

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..models.config import ModelConfig
from ..ops._native import native, use_native
from ..ops.activation import swiglu
from ..ops.embedding import embedding
from ..ops.attention import (flash_attention_fresh, flash_attention_paged, paged_decode,
                             rope_write_kv)
from ..ops.gemm import linear_nt, swiglu_linear_nt
from ..ops.norm import rms_norm
from ..ops.rope import rope_tables


# prefill of whole fresh prompts from the q|k|v rows instead of the paged cache (model_runner
# _execute); LUMEN_FRESH_PREFILL=0 always reads the cache
FRESH_PREFILL = os.environ.get("LUMEN_FRESH_PREFILL", "1") != "0"
# decode batches of at least this many rows run as two half-batches on two streams (TP = 1;
# 0 = off): ModelRunner._decode_split
DECODE_SPLIT_MIN = int(os.environ.get("LUMEN_DECODE_SPLIT", "0"))


@dataclass
class LayerW:
    ln1: torch.Tensor
    ln2: torch.Tensor
    qkv: torch.Tensor
    o: torch.Tensor
    gate_up: torch.Tensor
    down: torch.Tensor


class ServeWeights:
    """Inference weights extracted from a (LoRA-merged) LlamaForCausalLM, TP-sliced."""

    def __init__(self, model, tp_rank: int = 0, tp_size: int = 1):
        cfg: ModelConfig = model.config
        if cfg.arch != "llama":
            raise NotImplementedError("serving supports the Llama family")
        self.cfg = cfg
        nh, nkv, D, H, Fd = (cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim,
                             cfg.hidden_size, cfg.intermediate_size)
        if nh % tp_size or nkv % tp_size or Fd % tp_size:
            raise ValueError(f"TP={tp_size} must divide heads ({nh}/{nkv}) and FFN ({Fd})")
        self.nh, self.nkv = nh // tp_size, nkv // tp_size
        self.F = Fd // tp_size
        r = tp_rank
        qs, ks = nh * D, nkv * D
        lq, lk, lf = self.nh * D, self.nkv * D, self.F
        self.layers: List[LayerW] = []
        with torch.no_grad():
            for L in model.layers:
                W = L.self_attn.qkv_proj.weight
                qkv = torch.cat([W[r * lq:(r + 1) * lq], W[qs + r * lk:qs + (r + 1) * lk],
                                 W[qs + ks + r * lk:qs + ks + (r + 1) * lk]], 0).contiguous()
                o = L.self_attn.o_proj.weight[:, r * lq:(r + 1) * lq].contiguous()
                GU = L.mlp.gate_up_proj.weight
                gu = torch.cat([GU[r * lf:(r + 1) * lf], GU[Fd + r * lf:Fd + (r + 1) * lf]],
                               0).contiguous()
                dn = L.mlp.down_proj.weight[:, r * lf:(r + 1) * lf].contiguous()
                self.layers.append(LayerW(L.input_layernorm.weight, L.post_attention_layernorm.weight,
                                          qkv, o, gu, dn))
        self.embed = model.embed_tokens.weight
        self.norm = model.norm.weight
        # vocab-parallel LM head: each rank scores V/TP rows, logits all-gathered
        V = cfg.vocab_size
        self.vocab_shard = V // tp_size if V % tp_size == 0 else V
        lm = model.lm_head.weight
        self.lm_head = (lm[r * self.vocab_shard:(r + 1) * self.vocab_shard].contiguous()
                        if self.vocab_shard != V else lm)
        self.dtype = self.embed.dtype


@dataclass
class StepInput:
    kind: str                          # mixed | decode
    tokens: torch.Tensor               # [T] int64 (device): prefill chunk rows, then decode rows
    positions: torch.Tensor            # [T] int32
    slots: torch.Tensor                # [T] int64
    cu_seqlens: List[int]              # prefill chunks: per-sequence row offsets (host), [0] if none
    block_tables: Optional[torch.Tensor] = None  # decode rows [N, maxb] int32
    context_lens: Optional[torch.Tensor] = None  # decode rows [N] int32
    max_context: int = 0
    lora_ids: Optional[torch.Tensor] = None      # [T] int32 adapter slot per token (multi-LoRA)
    kv_lens: Optional[List[int]] = None          # prefill chunks: cached context + chunk (host)
    kv_lens_t: Optional[torch.Tensor] = None     # ... on the device, int32 [P]
    prefill_tables: Optional[torch.Tensor] = None  # prefill chunks [P, maxb] int32
    sample_rows: Optional[torch.Tensor] = None   # rows whose logits are sampled, int64 [R]
    temps: Optional[torch.Tensor] = None         # [R] f32 sampling temperature per sampled row
    top_ps: Optional[torch.Tensor] = None        # [R] f32
    top_ks: Optional[torch.Tensor] = None        # [R] int32
    extra_rows: Optional[torch.Tensor] = None    # prompt-logprob rows (TP = 1), int64 [E]
    prompt_meta: Optional[list] = None           # host: (seq, first scored token, count, row)

    @property
    def num_prefill_rows(self) -> int:
        return self.cu_seqlens[-1] if self.cu_seqlens else 0




def kv_bytes_per_token(cfg: ModelConfig, dtype_bytes: int = 2, tp_size: int = 1) -> int:
    return 2 * cfg.num_hidden_layers * (cfg.num_key_value_heads // tp_size) * cfg.head_dim * dtype_bytes


class ModelRunner:
    def __init__(self, weights: ServeWeights, num_blocks: int, block_size: int,
                 device: torch.device, max_model_len: int = 4096, tp_group=None,
                 use_graphs: bool = True, max_graph_batch: int = 256, custom_ar=None,
                 kv_dtype: Optional[torch.dtype] = None):
        self.w = weights
        self.cfg = weights.cfg
        self.device = device
        self.block_size = block_size
        self.num_blocks = num_blocks
        self.max_model_len = max_model_len
        self.tp_group = tp_group
        self.tp = dist.get_world_size(tp_group) if tp_group is not None else 1
        cfg = self.cfg
        D = cfg.head_dim
        self.q_size, self.kv_size = self.w.nh * D, self.w.nkv * D
        self.max_blocks = (max_model_len + block_size - 1) // block_size
        dt = weights.dtype
        # KV-cache element type: the model dtype, or fp8 e4m3 (vLLM --kv-cache-dtype fp8: half
        # the K/V bytes every decode step streams)
        self.kv_dtype = kv_dtype or dt
        self.k_cache = [torch.zeros(num_blocks, self.w.nkv, block_size, D, dtype=self.kv_dtype,
                                    device=device)
                        for _ in range(cfg.num_hidden_layers)]
        self.v_cache = [torch.zeros_like(k) for k in self.k_cache]
        self.cos, self.sin = rope_tables(D, max(cfg.max_position_embeddings, max_model_len),
                                         cfg.rope_theta, device)
        self.scale = 1.0 / math.sqrt(D)
        # TP: row-parallel sums go through the custom all-reduce (IPC peer memory, one kernel,
        # graph-capturable) when it is up; RCCL otherwise (and then decode runs eagerly)
        self.car = custom_ar
        self.use_graphs = (use_graphs and device.type == "cuda"
                           and (self.tp == 1 or self.car is not None))
        buckets = [b for b in (1, 2, 4, 8, 16, 32, 64, 96, 128, 160, 192, 224, 256)
                   if b <= max_graph_batch]
        if self.tp > 1 and self.car is not None:
            # a captured bucket may only hold custom all-reduces (RCCL cannot be captured)
            row_bytes = cfg.hidden_size * torch.empty((), dtype=dt).element_size()
            buckets = [b for b in buckets if b * row_bytes <= self.car.max_bytes]
        self.graph_buckets = buckets
        self.use_graphs = self.use_graphs and bool(buckets)
        # the vocab gather joins the graph when every bucket's logits shard fits the staging
        # buffer (then a decode step is one graph replay; otherwise an RCCL gather follows it)
        self._graph_gathers = self.tp == 1 or self.w.vocab_shard == cfg.vocab_size or (
            self.car is not None and self.w.vocab_shard % 8 == 0
            and max(buckets or [1]) * self.w.vocab_shard * torch.empty((), dtype=dt).element_size()
            <= self.car.max_bytes)
        self._graphs: Dict[int, tuple] = {}
        self._graph_pool = None
        # context tokens per decode workgroup at full batch (LUMEN_PA_PARTITION): 2048 measured
        # 20.15 vs 20.87 ms ITL at 256 requests (one partition per sequence: no partials, no
        # merge kernel); the single-pass kernel keeps no per-token scores, so long partitions
        # cost no LDS
        self.partition = int(os.environ.get("LUMEN_PA_PARTITION", "2048"))
        self.lora = None  # serve.multi_lora.MultiLoRA when adapters are served un-merged

    # ------------------------------------------------------------------------------------------
    def check_collectives(self) -> None:
        """Raise if a TP custom all-reduce / all-gather timed out waiting for a peer (reads a
        pinned host word: call after the step's host sync)."""
        if self.car is not None:
            self.car.poll()

    def _allreduce(self, x):
        if self.tp > 1:
            if self.car is not None and self.car.prefer(x):
                self.car.all_reduce(x)
            else:
                dist.all_reduce(x, group=self.tp_group)
        return x

    def _layers(self, h, positions, slots, attn_fn, lora_ids=None, mark=None):
        cfg = self.cfg
        res = None
        T = h.shape[0]
        D = cfg.head_dim
        ml = self.lora if lora_ids is not None else None
        masks = {n: ml.mask(lora_ids, n) for n in (1, 2, 3)} if ml is not None else None
        for i, L in enumerate(self.w.layers):
            y, res = rms_norm(h, L.ln1, cfg.rms_norm_eps, res)
            qkv = linear_nt(y, L.qkv)
            if mark is not None and i == 0:
                mark.record()   # split decode: the second half starts here
            if ml is not None:
                ml.apply(i, "qkv", y, qkv, masks)
            rope_write_kv(qkv, positions, self.w.nh, self.w.nkv, D, self.cos, self.sin,
                          self.k_cache[i], self.v_cache[i], slots)
            o = attn_fn(qkv, i)
            a = self._allreduce(linear_nt(o, L.o))
            if ml is not None:
                ml.apply(i, "o", o, a, masks, self._allreduce)
            y2, res = rms_norm(a, L.ln2, cfg.rms_norm_eps, res)
            gu = linear_nt(y2, L.gate_up)
            if ml is not None:
                ml.apply(i, "gate_up", y2, gu, masks)
            if ml is None:  # SwiGLU kernel + down projection (GEMV at batch <= 4)
                h = self._allreduce(swiglu_linear_nt(gu, L.down))
            else:
                act = swiglu(gu)
                h = self._allreduce(linear_nt(act, L.down))
                ml.apply(i, "down", act, h, masks, self._allreduce)
        return h, res

    def _vocab_gather(self, logits):
        """[R, V/TP] local logits -> [R, V] on every rank (vocab-parallel LM head)."""
        if self.tp == 1 or self.w.vocab_shard == self.cfg.vocab_size:
            return logits
        R, Vs = logits.shape
        if self.car is not None and self.car.gather_eligible(logits):
            return self.car.all_gather_cols(logits.contiguous())
        if logits.is_cuda:
            buf = torch.empty(self.tp, R, Vs, dtype=logits.dtype, device=logits.device)
            dist.all_gather_into_tensor(buf, logits.contiguous(), group=self.tp_group)
            parts = buf.unbind(0)
        else:
            parts = [torch.empty_like(logits) for _ in range(self.tp)]
            dist.all_gather(parts, logits.contiguous(), group=self.tp_group)
        return torch.cat(parts, 1)

    def _logits(self, h, res, rows, extra=None):
        if extra is not None and extra.numel():
            # prompt scoring rows (TP = 1): their logits are left in ``extra_logits``
            y, _ = rms_norm(h[extra], self.w.norm, self.cfg.rms_norm_eps, res[extra])
            self.extra_logits = torch.matmul(y, self.w.lm_head.t())
        if rows.numel() == 0:  # a chunk that completes no prompt samples nothing
            return torch.empty(0, self.cfg.vocab_size, device=h.device, dtype=h.dtype)
        y, _ = rms_norm(h[rows], self.w.norm, self.cfg.rms_norm_eps, res[rows])
        return self._vocab_gather(torch.matmul(y, self.w.lm_head.t()))

    # ---- mixed step: prefill chunks (whole prompts or pieces of long ones) + decode rows -----
    @torch.no_grad()
    def execute(self, inp: StepInput) -> torch.Tensor:
        """Logits [len(sample_rows), V] of one mixed step (see StepInput): prefill chunk and
        decode rows in ONE forward (every weight read once for both).  (Running the decode rows
        as their graph on a second stream concurrently with the chunk measured worse: 7.46k vs
        7.55k tok/s and ITL p99 64 vs 40 ms at 256 x 512 / 128, profiles/r3_serve -- the chunk's
        GEMMs already fill the chip, and the decode rows then waited for a full-budget chunk.)"""
        return self._execute(inp)

    def _execute(self, inp: StepInput) -> torch.Tensor:
        h = embedding(inp.tokens, self.w.embed)
        T = inp.tokens.shape[0]
        Tp = inp.num_prefill_rows
        N = T - Tp
        cu = inp.cu_seqlens
        nh, nkv, D = self.w.nh, self.w.nkv, self.cfg.head_dim

        # every chunk a whole fresh prompt (no cached context): attention straight from the
        # rotated q|k|v rows, as in training (the paged kernel re-reads K/V through the block
        # tables: 65 vs 42 us per layer for 8 x 512 tokens; with an fp8 cache it also skips the
        # block dequantisation)
        fresh = (FRESH_PREFILL and Tp > 0 and h.is_cuda and use_native(h) and D == 128
                 and inp.kv_lens is not None
                 and all(int(kl) == cu[j + 1] - cu[j] for j, kl in enumerate(inp.kv_lens)))

        def attn(qkv, i):
            o = torch.empty(T, nh * D, device=qkv.device, dtype=qkv.dtype)
            if Tp and fresh:
                flash_attention_fresh(qkv[:Tp], cu, nh, nkv, D, self.scale, out=o[:Tp])
            elif Tp:
                # this chunk's K/V are already in the cache (rope_write_kv): read everything the
                # chunk may see -- cached context + chunk -- from there
                flash_attention_paged(qkv[:Tp], self.k_cache[i], self.v_cache[i], cu,
                                      inp.kv_lens_t if qkv.is_cuda else inp.kv_lens,
                                      inp.prefill_tables, nh, nkv, D, self.scale, out=o[:Tp])
            if N:
                q = qkv[Tp:, :self.q_size].reshape(N, nh, D)
                o[Tp:] = paged_decode(q, self.k_cache[i], self.v_cache[i], inp.block_tables,
                                      inp.context_lens, inp.max_context, self.scale,
                                      self.decode_partition(N)).view(N, nh * D)
            return o

        h, res = self._layers(h, inp.positions, inp.slots, attn, inp.lora_ids)
        return self._logits(h, res, inp.sample_rows, inp.extra_rows)

    prefill = execute  # a whole-prompt step is a mixed step without decode rows

    # ---- decode: one token per sequence ----------------------------------------------------
    def _split_ok(self, N: int, lora_ids) -> bool:
        return (DECODE_SPLIT_MIN > 0 and N >= DECODE_SPLIT_MIN and N % 32 == 0 and self.tp == 1
                and lora_ids is None and self.device.type == "cuda")

    def _decode_eager(self, tokens, positions, slots, block_tables, context_lens, max_context,
                      lora_ids=None, gather: bool = True):
        N = tokens.shape[0]
        if self._split_ok(N, lora_ids):
            return self._decode_split(tokens, positions, slots, block_tables, context_lens,
                                      max_context)
        return self._decode_rows(tokens, positions, slots, block_tables, context_lens,
                                 max_context, lora_ids, gather)

    def _decode_split(self, tokens, positions, slots, block_tables, context_lens, max_context):
        """Two half-batches on two streams (TP = 1, N >= DECODE_SPLIT_MIN): the halves are
        independent (own rows, own K/V slots), so while one half's paged attention streams its
        K/V (HBM-bound) the other half's projection GEMMs (latency / L2-bound at these M) run
        beside it.  The second half starts after the first half's first q|k|v projection, so
        the two settle half a layer apart.  Costs one more read of the weights per step.
        Captured in the decode graph like the single-stream path (fork / join by events).
        Measured NEGATIVE on Llama-2-7B at 256 rows x ~600 context (profiles/r5_decode):
        21.1-21.2 vs 19.55 ms per step -- side by side the halves' paged attention ran at 222 us
        per 128-row call (444 per layer vs 400 alone) and the M = 128 projections cost 9.2 ms
        per step for both halves, so the overlap never paid for the doubled weight reads.  Off
        by default (LUMEN_DECODE_SPLIT=0)."""
        N = tokens.shape[0]
        hN = N // 2
        cur = torch.cuda.current_stream(self.device)
        side = getattr(self, "_split_stream", None)
        if side is None:
            side = self._split_stream = torch.cuda.Stream(device=self.device)
        first = torch.cuda.Event()
        self._split_mark = first
        outs = [None, None]
        a = slice(0, hN)
        outs[0] = self._decode_rows(tokens[a], positions[a], slots[a], block_tables[a],
                                    context_lens[a], max_context, None, True, mark=first)
        side.wait_event(first)
        with torch.cuda.stream(side):
            b = slice(hN, N)
            outs[1] = self._decode_rows(tokens[b], positions[b], slots[b], block_tables[b],
                                        context_lens[b], max_context, None, True)
        cur.wait_stream(side)
        return torch.cat(outs, 0)

    def _decode_rows(self, tokens, positions, slots, block_tables, context_lens, max_context,
                     lora_ids=None, gather: bool = True, mark=None):
        h = embedding(tokens, self.w.embed)
        N = tokens.shape[0]
        nh, D = self.w.nh, self.cfg.head_dim

        def attn(qkv, i):
            q = qkv[:, :self.q_size].reshape(N, nh, D)
            return paged_decode(q, self.k_cache[i], self.v_cache[i], block_tables, context_lens,
                                max_context, self.scale, self.decode_partition(N)).view(N, nh * D)

        h, res = self._layers(h, positions, slots, attn, lora_ids, mark=mark)
        y, _ = rms_norm(h, self.w.norm, self.cfg.rms_norm_eps, res)
        logits = linear_nt(y, self.w.lm_head)
        return self._vocab_gather(logits) if gather else logits

    def decode_partition(self, n_seqs: int) -> int:
        """Context tokens per paged-decode workgroup for a batch of ``n_seqs``: the full-batch
        partition (2048) once sequences x kv heads x partitions give >= 2048 workgroups (8 per
        CU), shorter partitions (down to 64) below that, so a small batch still spreads its KV
        read over the chip (batch 1 at 576 tokens of context: 64 -> 288 workgroups; the kernel
        went from 53 to a few us)."""
        pairs = max(1, n_seqs * self.w.nkv)
        part = self.partition
        while part > 64 and pairs * (self.partition // part) < 2048:
            part //= 2
        return part

    @torch.no_grad()
    def decode(self, inp: StepInput) -> torch.Tensor:
        N = inp.tokens.shape[0]
        if not self.use_graphs or N > self.graph_buckets[-1]:
            return self._decode_eager(inp.tokens, inp.positions, inp.slots, inp.block_tables,
                                      inp.context_lens, inp.max_context, inp.lora_ids)
        bucket = next(b for b in self.graph_buckets if b >= N)
        g = self._graphs.get(bucket)
        if g is None:
            g = self._capture(bucket)
        graph, st, out = g
        st["tokens"][:N].copy_(inp.tokens)
        st["positions"][:N].copy_(inp.positions)
        st["slots"][:N].copy_(inp.slots)
        nb = inp.block_tables.shape[1]
        st["block_tables"][:N, :nb].copy_(inp.block_tables)
        st["context_lens"][:N].copy_(inp.context_lens)
        if self.lora is not None:
            st["lora_ids"][:N].copy_(inp.lora_ids)
        if N < bucket:  # padding rows: no cache write, one-token context on block 0
            st["slots"][N:].fill_(-1)
            st["context_lens"][N:].fill_(1)
        graph.replay()
        if self._graph_gathers:
            return out[:N]
        # the vocab-parallel gather stays outside the graph when it would need RCCL
        return self._vocab_gather(out[:N])

    def _capture(self, bucket: int):
        dev = self.device
        st = {"tokens": torch.zeros(bucket, dtype=torch.long, device=dev),
              "positions": torch.zeros(bucket, dtype=torch.int32, device=dev),
              "slots": torch.full((bucket,), -1, dtype=torch.long, device=dev),
              "block_tables": torch.zeros(bucket, self.max_blocks, dtype=torch.int32, device=dev),
              "context_lens": torch.ones(bucket, dtype=torch.int32, device=dev)}
        if self.lora is not None:
            st["lora_ids"] = torch.zeros(bucket, dtype=torch.int32, device=dev)
        args = (st["tokens"], st["positions"], st["slots"], st["block_tables"],
                st["context_lens"], self.max_model_len, st.get("lora_ids"), self._graph_gathers)
        # one warm-up stream for every bucket (per-stream decode-GEMM workspaces stay few)
        s = getattr(self, "_warm_stream", None)
        if s is None:
            s = self._warm_stream = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up (allocator, hipBLASLt heuristics) outside capture
                self._decode_eager(*args)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(graph, pool=self._graph_pool):
            out = self._decode_eager(*args)
        self._graphs[bucket] = (graph, st, out)
        return self._graphs[bucket]

    # ---- sampling ----------------------------------------------------------------------------
    @torch.no_grad()
    def sample(self, logits: torch.Tensor, temps: Seq[float], top_ps: Seq[float],
               top_ks: Seq[int], seed: int, offset: int, want_logprobs: bool = True):
        R = logits.shape[0]
        dev = logits.device
        # device tensors (the engine ships them in its packed step copy); lists are converted
        # here with a blocking copy
        t = temps if torch.is_tensor(temps) else torch.tensor(temps, dtype=torch.float32, device=dev)
        p = top_ps if torch.is_tensor(top_ps) else torch.tensor(top_ps, dtype=torch.float32,
                                                                device=dev)
        k = top_ks if torch.is_tensor(top_ks) else torch.tensor(top_ks, dtype=torch.int32, device=dev)
        if use_native(logits):
            out = torch.empty(R, dtype=torch.long, device=dev)
            lp = torch.empty(R, dtype=torch.float32, device=dev) if want_logprobs else None
            native().sample(logits.contiguous(), t, p, k, seed, offset, out, lp)
            return out, lp
        return sample_ref(logits, t, p, k, seed, offset)


def topk_topp_keep(zs: torch.Tensor, k: int, p: float) -> torch.Tensor:
    """The kept set of vLLM 0.6.0's ``_apply_top_k_top_p`` for one row of scaled logits: top-k
    keeps every value >= the k-th largest (ties kept); top-p then keeps the smallest head of
    the sorted top-k-renormalised distribution whose mass reaches p (at least one token)."""
    V = zs.shape[-1]
    keep = torch.ones(V, dtype=torch.bool, device=zs.device)
    if 0 < k < V:
        keep &= zs >= torch.topk(zs, k).values[-1]
    if p < 1.0:
        zk = torch.where(keep, zs, torch.full_like(zs, -float("inf")))
        sp, idx = torch.sort(torch.softmax(zk, -1), descending=True)
        c = torch.cumsum(sp, 0)
        cut = int((c - sp < p).sum())  # tokens whose mass strictly above them is < p
        m = torch.zeros(V, dtype=torch.bool, device=zs.device)
        m[idx[:max(cut, 1)]] = True
        keep &= m
    return keep


def sample_ref(logits, temps, top_ps, top_ks, seed, offset):
    """Torch sampler (CPU path): same semantics as kernels/sampling.hip, torch RNG."""
    R, V = logits.shape
    g = torch.Generator(device=logits.device).manual_seed((seed * 1000003 + offset) & 0x7FFFFFFF)
    out = torch.empty(R, dtype=torch.long, device=logits.device)
    lps = torch.empty(R, dtype=torch.float32, device=logits.device)
    for i in range(R):
        z = logits[i].float()
        T = float(temps[i])
        if T <= 0:
            tok = int(z.argmax())
            zs = z
        else:
            zs = z / T
            keep = topk_topp_keep(zs, int(top_ks[i]), float(top_ps[i]))
            probs = torch.softmax(zs, -1)
            pr = torch.where(keep, probs, torch.zeros_like(probs))
            tok = int(torch.multinomial(pr / pr.sum(), 1, generator=g))
        out[i] = tok
        lps[i] = torch.log_softmax(zs, -1)[tok]
    return out, lps
