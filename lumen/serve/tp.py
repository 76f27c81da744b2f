"""Tensor-parallel serving plumbing: step broadcast from rank 0 and the worker loop.

Each step travels in two parts (no pickled Python objects on the hot path):

* a HOST header over the host (gloo) group -- kind, the shape integers every rank needs to pick
  its graph bucket / kernel launch sizes, and the prefill chunks' ``cu_seqlens`` / ``kv_lens``
  (launch parameters of the paged prefill kernel): a fixed-size CPU int64 message, host to host;
* the DEVICE payload (tokens | positions | slots | prefill kv lens / block tables | decode
  block tables / context lens | sampled rows | LoRA slots) as ONE int64 RCCL broadcast straight
  into a device buffer, stream-ordered after the previous step.

A worker never reads device memory on the host: it builds the StepInput as views of the
payload and replays the decode graph (or runs the mixed step) as soon as the header arrives, so
its host runs ahead of its GPU exactly like rank 0's with async scheduling.  (Until round 3 the
header rode in the device message and the worker's ``msg[:10].tolist()`` synchronised its host
with its GPU once per step.)  The row-parallel all-reduces inside the layers keep the ranks in
lock-step on the devices.
"""
from __future__ import annotations

import os
import random
import time
from typing import Optional

import torch
import torch.distributed as dist

from ..parallel.dist import host_group
from .model_runner import StepInput

KIND = {"mixed": 0, "decode": 1, "shutdown": 2}
HDR = 12  # kind, T, P, maxb_p, N, maxb_d, max_context, R, lora, payload numel, -, -
HOST_CAP = 1024  # cu_seqlens + kv_lens values carried inline with the host header


def _host_bcast(t: torch.Tensor) -> None:
    dist.broadcast(t, src=0, group=host_group())


# fault injection (tests): LUMEN_TP_INJECT_DELAY_MS=N makes every rank sleep a pseudo-random
# 0..N ms at each protocol point (between header and payload on both sides, before a worker
# launches its step), so ranks drift apart on the host the way a loaded box makes them
_DELAY_MS = float(os.environ.get("LUMEN_TP_INJECT_DELAY_MS", "0") or 0)
_rng = random.Random(int(os.environ.get("RANK", "0")) * 7919 + 1)


def _inject_delay() -> None:
    if _DELAY_MS > 0:
        time.sleep(_rng.random() * _DELAY_MS / 1000.0)


def pack_step(inp: Optional[StepInput], device) -> None:
    hdr = torch.zeros(HDR + HOST_CAP, dtype=torch.long)
    if inp is None:
        hdr[0] = KIND["shutdown"]
        _host_bcast(hdr)
        return
    T = inp.tokens.numel()
    P = len(inp.cu_seqlens) - 1
    parts = [inp.tokens.long(), inp.positions.long(), inp.slots.long()]
    maxb_p = N = maxb_d = 0
    host = []
    if P:
        maxb_p = inp.prefill_tables.shape[1]
        host = list(inp.cu_seqlens) + list(inp.kv_lens)
        parts += [inp.kv_lens_t.long(), inp.prefill_tables.long().reshape(-1)]
    if inp.block_tables is not None:
        N, maxb_d = inp.block_tables.shape
        parts += [inp.block_tables.long().reshape(-1), inp.context_lens.long()]
    R = inp.sample_rows.numel()
    parts.append(inp.sample_rows.long())
    if inp.lora_ids is not None:  # multi-LoRA: per-token adapter slots ride at the end
        parts.append(inp.lora_ids.long())
    payload = torch.cat([p.to(device) for p in parts])
    n = payload.numel()
    hdr[:10] = torch.tensor([KIND[inp.kind], T, P, maxb_p, N, maxb_d, inp.max_context, R,
                             int(inp.lora_ids is not None), n])
    k = min(len(host), HOST_CAP)
    if k:
        hdr[HDR:HDR + k] = torch.tensor(host[:k], dtype=torch.long)
    _host_bcast(hdr)
    if len(host) > HOST_CAP:
        _host_bcast(torch.tensor(host[HOST_CAP:], dtype=torch.long))
    _inject_delay()
    dist.broadcast(payload, src=0)


def recv_step(device) -> Optional[StepInput]:
    hdr = torch.empty(HDR + HOST_CAP, dtype=torch.long)
    _host_bcast(hdr)
    kind, T, P, maxb_p, N, maxb_d, maxc, R, has_lora, n = hdr[:10].tolist()
    if kind == KIND["shutdown"]:
        return None
    host = []
    if P:
        nh = 2 * P + 1
        host = hdr[HDR:HDR + min(nh, HOST_CAP)].tolist()
        if nh > HOST_CAP:
            rest = torch.empty(nh - HOST_CAP, dtype=torch.long)
            _host_bcast(rest)
            host += rest.tolist()
    payload = torch.empty(n, dtype=torch.long, device=device)
    _inject_delay()
    dist.broadcast(payload, src=0)
    inp = StepInput("mixed" if kind == KIND["mixed"] else "decode", payload[:T],
                    payload[T:2 * T].int(), payload[2 * T:3 * T], [0])
    o = 3 * T
    if P:
        inp.cu_seqlens = host[:P + 1]
        inp.kv_lens = host[P + 1:2 * P + 1]
        inp.kv_lens_t = payload[o:o + P].int()
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
    """Ranks 1..TP-1: execute broadcast steps until shutdown.  The host blocks only on rank 0's
    host header, never on this rank's GPU."""
    while True:
        inp = recv_step(runner.device)
        runner.check_collectives()   # a pinned host word: no device sync
        if inp is None:
            return
        _inject_delay()
        if inp.kind == "decode":
            runner.decode(inp)
        else:
            runner.execute(inp)
