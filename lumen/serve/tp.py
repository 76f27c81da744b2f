"""Tensor-parallel serving plumbing: step broadcast from rank 0 and the worker loop.

Rank 0 (scheduler + API) sends each step as ONE fixed-size int64 broadcast: a 12-int64 header
followed by the payload (tokens | positions | slots | prefill cu / kv lens / block tables |
decode block tables / context lens | sampled rows | LoRA slots) -- no pickled Python objects on
the hot path.  A payload larger than the inline capacity (CAP, 16384 values: a
256-sequence decode step with ~40 blocks per sequence fits) sends its remainder in a second
broadcast.  Workers rebuild the StepInput and run the same model step; the row-parallel
all-reduces inside the layers keep the ranks in lock-step.  With async scheduling (default)
rank 0 broadcasts a step when it LAUNCHES it, decode tokens straight from the device.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .model_runner import StepInput

KIND = {"mixed": 0, "decode": 1, "shutdown": 2}
HDR = 12  # kind, T, P, maxb_p, N, maxb_d, max_context, R, lora, payload numel, -, -
CAP = 16384  # payload values carried inline with the header


def pack_step(inp: Optional[StepInput], device) -> None:
    if inp is None:
        msg = torch.zeros(HDR + CAP, dtype=torch.long, device=device)
        msg[0] = KIND["shutdown"]
        dist.broadcast(msg, src=0)
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
    n = payload.numel()
    hdr = torch.tensor([KIND[inp.kind], T, P, maxb_p, N, maxb_d, inp.max_context, R,
                        int(inp.lora_ids is not None), n, 0, 0], dtype=torch.long)
    msg = torch.zeros(HDR + CAP, dtype=torch.long, device=device)
    msg[:HDR].copy_(hdr, non_blocking=False)
    msg[HDR:HDR + min(n, CAP)] = payload[:CAP]
    dist.broadcast(msg, src=0)
    if n > CAP:
        dist.broadcast(payload[CAP:].contiguous(), src=0)


def recv_step(device) -> Optional[StepInput]:
    msg = torch.empty(HDR + CAP, dtype=torch.long, device=device)
    dist.broadcast(msg, src=0)
    kind, T, P, maxb_p, N, maxb_d, maxc, R, has_lora, n = msg[:10].tolist()
    if kind == KIND["shutdown"]:
        return None
    if n <= CAP:
        payload = msg[HDR:HDR + n]
    else:
        rest = torch.empty(n - CAP, dtype=torch.long, device=device)
        dist.broadcast(rest, src=0)
        payload = torch.cat([msg[HDR:], rest])
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
