"""Tensor-parallel serving plumbing: step broadcast from rank 0 and the worker loop.

Rank 0 (scheduler + API) sends each step as a fixed 12-int64 header and one int64 payload
(tokens | positions | slots | prefill cu / kv lens / block tables | decode block tables /
context lens | sampled rows | LoRA slots) with two RCCL
broadcasts -- no pickled Python objects on the hot path.  Workers rebuild the
StepInput and run the same model step; the row-parallel all-reduces inside the layers keep the
ranks in lock-step.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .model_runner import StepInput

KIND = {"mixed": 0, "decode": 1, "shutdown": 2}
HDR = 12  # kind, T, P, maxb_p, N, maxb_d, max_context, R, lora, payload numel, -, -


def pack_step(inp: Optional[StepInput], device) -> None:
    hdr = torch.zeros(HDR, dtype=torch.long, device=device)
    if inp is None:
        hdr[0] = KIND["shutdown"]
        dist.broadcast(hdr, src=0)
        return
    T = inp.tokens.numel()
    P = len(inp.cu_seqlens) - 1
    parts = [inp.tokens.long(), inp.positions.long(), inp.slots.long()]
    maxb_p = N = maxb_d = 0
    if P:
        maxb_p = inp.prefill_tables.shape[1]
        parts += [torch.tensor(inp.cu_seqlens, dtype=torch.long, device=device),
                  inp.kv_lens_t.long(), inp.prefill_tables.long().reshape(-1)]
    if inp.block_tables is not None:
        N, maxb_d = inp.block_tables.shape
        parts += [inp.block_tables.long().reshape(-1), inp.context_lens.long()]
    R = inp.sample_rows.numel()
    parts.append(inp.sample_rows.long())
    if inp.lora_ids is not None:  # multi-LoRA: per-token adapter slots ride at the end
        parts.append(inp.lora_ids.long())
    payload = torch.cat(parts)
    hdr[:10] = torch.tensor([KIND[inp.kind], T, P, maxb_p, N, maxb_d, inp.max_context, R,
                             int(inp.lora_ids is not None), payload.numel()])
    dist.broadcast(hdr, src=0)
    dist.broadcast(payload, src=0)


def recv_step(device) -> Optional[StepInput]:
    hdr = torch.zeros(HDR, dtype=torch.long, device=device)
    dist.broadcast(hdr, src=0)
    kind, T, P, maxb_p, N, maxb_d, maxc, R, has_lora, n = hdr.tolist()[:10]
    if kind == KIND["shutdown"]:
        return None
    payload = torch.empty(n, dtype=torch.long, device=device)
    dist.broadcast(payload, src=0)
    inp = StepInput("mixed" if kind == KIND["mixed"] else "decode", payload[:T],
                    payload[T:2 * T].int(), payload[2 * T:3 * T], [0])
    o = 3 * T
    if P:
        inp.cu_seqlens = payload[o:o + P + 1].tolist()
        o += P + 1
        inp.kv_lens_t = payload[o:o + P].int()
        inp.kv_lens = inp.kv_lens_t.tolist()
        o += P
        inp.prefill_tables = payload[o:o + P * maxb_p].view(P, maxb_p).int()
        o += P * maxb_p
    if N:
        inp.block_tables = payload[o:o + N * maxb_d].view(N, maxb_d).int()
        o += N * maxb_d
        inp.context_lens = payload[o:o + N].int()
        o += N
        inp.max_context = maxc
    inp.sample_rows = payload[o:o + R]
    o += R
    if has_lora:
        inp.lora_ids = payload[o:o + T].int()
    return inp


def worker_loop(runner) -> None:
    """Ranks 1..TP-1: execute broadcast steps until shutdown."""
    while True:
        inp = recv_step(runner.device)   # host-syncs: the previous step has completed
        runner.check_collectives()
        if inp is None:
            return
        if inp.kind == "decode":
            runner.decode(inp)
        else:
            runner.execute(inp)
