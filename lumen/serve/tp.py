"""Tensor-parallel serving plumbing: step broadcast from rank 0 and the worker loop.

Rank 0 (scheduler + API) sends each step as a fixed 8-int64 header and one int64 payload
(tokens | positions | slots | cu_seqlens | block tables | context lens) with two RCCL
broadcasts -- no pickled Python objects on the hot path.  Workers rebuild the
StepInput and run the same model step; the row-parallel all-reduces inside the layers keep the
ranks in lock-step.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .model_runner import StepInput

KIND = {"prefill": 0, "decode": 1, "shutdown": 2}


def pack_step(inp: Optional[StepInput], device) -> None:
    hdr = torch.zeros(8, dtype=torch.long, device=device)
    if inp is None:
        hdr[0] = KIND["shutdown"]
        dist.broadcast(hdr, src=0)
        return
    T = inp.tokens.numel()
    parts = [inp.tokens.long(), inp.positions.long(), inp.slots.long()]
    if inp.kind == "prefill":
        cu = torch.tensor(inp.cu_seqlens, dtype=torch.long, device=device)
        parts.append(cu)
        hdr[:4] = torch.tensor([KIND["prefill"], T, len(inp.cu_seqlens), 0])
    else:
        N, nb = inp.block_tables.shape
        parts += [inp.block_tables.long().reshape(-1), inp.context_lens.long()]
        hdr[:5] = torch.tensor([KIND["decode"], T, N, nb, inp.max_context])
    if inp.lora_ids is not None:  # multi-LoRA: per-token adapter slots ride at the end
        parts.append(inp.lora_ids.long())
        hdr[5] = 1
    payload = torch.cat(parts)
    hdr[7] = payload.numel()
    dist.broadcast(hdr, src=0)
    dist.broadcast(payload, src=0)


def recv_step(device) -> Optional[StepInput]:
    hdr = torch.zeros(8, dtype=torch.long, device=device)
    dist.broadcast(hdr, src=0)
    h = hdr.tolist()
    if h[0] == KIND["shutdown"]:
        return None
    payload = torch.empty(h[7], dtype=torch.long, device=device)
    dist.broadcast(payload, src=0)
    T = h[1]
    tok, pos, slots = payload[:T], payload[T:2 * T].int(), payload[2 * T:3 * T]
    rest = payload[3 * T:]
    lora = payload[-T:].int() if h[5] else None
    if h[0] == KIND["prefill"]:
        cu = rest[:h[2]].tolist()
        return StepInput("prefill", tok, pos, slots, cu, lora_ids=lora)
    N, nb, maxc = h[2], h[3], h[4]
    bt = rest[:N * nb].view(N, nb).int()
    cl = rest[N * nb:N * nb + N].int()
    return StepInput("decode", tok, pos, slots, [], bt, cl, maxc, lora_ids=lora)


def worker_loop(runner) -> None:
    """Ranks 1..TP-1: execute broadcast steps until shutdown."""
    while True:
        inp = recv_step(runner.device)   # host-syncs: the previous step has completed
        runner.check_collectives()
        if inp is None:
            return
        if inp.kind == "prefill":
            runner.prefill(inp)
        else:
            runner.decode(inp)
