"""Projection GEMMs for decode: y = x @ W^T.

At decode batch 1-4 the projection is a pure stream of the weight matrix; for the shapes where it
measured faster the HIP weight-streaming kernel (``kernels/skinny_gemm.hip``) runs it instead
of a library GEMM.  Larger batches (and CPU tensors) go to ``torch.matmul`` (hipBLASLt with the
tuned table)."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ._native import native, use_native

# Measured per shape against hipBLASLt with the tuned table (lumen/bench/skinny_bench.py
# --m1-forms, profiles/r02_serve/m1_forms.jsonl): the rows-per-lane weight-streaming kernel
# reaches 4.3-6.5 TB/s at M = 1 and beats hipBLASLt at every Llama-2-7B projection (qkv 17.0 vs
# 22.9 us, o 7.8 vs 22.7, gate_up 27.8 vs 37.3, down 16.5 vs 27.5, lm_head 38.4 vs 60.6); at
# M = 2 it still wins or ties everywhere (o 10.4 vs 22.6, down 20.7 vs 27.6, lm_head 51.4 vs
# 59.0); at M = 3-4 only the N = 4096 projections (o, down) stay ahead, and from M = 5 on
# hipBLASLt wins, so those are library GEMMs.
SKINNY_MAX_M = int(os.environ.get("LUMEN_SKINNY_MAX_M", "4"))
SKINNY_MAX_N = int(os.environ.get("LUMEN_SKINNY_MAX_N", str(1 << 30)))
SKINNY_WIDE_MAX_M = 2  # above this M only N <= 4096 projections take the GEMV


def skinny_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (0 < x.shape[0] <= min(SKINNY_MAX_M, 16) and w.shape[0] <= SKINNY_MAX_N
            and (x.shape[0] <= SKINNY_WIDE_MAX_M or w.shape[0] <= 4096)
            and use_native(x) and x.dim() == 2
            and w.dim() == 2 and x.dtype == w.dtype and x.dtype in (torch.bfloat16, torch.float16)
            and x.stride(1) == 1 and w.is_contiguous() and x.shape[1] == w.shape[1]
            and (w.shape[0] % 4 == 0 and w.shape[1] % 8 == 0 and x.stride(0) % 8 == 0
                 if x.shape[0] <= 4 else w.shape[0] % 16 == 0 and w.shape[1] % 128 == 0))


# Decode batches 5..256: the decode-batch MFMA GEMM (kernels/decode_gemm.hip) where the measured
# plan table (configs/kernels/decode_gemm_plans.json, written by lumen/bench/decode_gemm_probe.py) has
# a winning (BM, BN, split-K) for the shape, hipBLASLt with the tuned table otherwise.  (Two
# earlier hand-written attempts lost, scripts/probes/: 32-row M tiles, and all-M-rows tiles over
# all of K whose every workgroup pulled the whole x through its CU's load path.)
DG_BMS = (64, 128, 192, 256)
DG_BNS = {256: (64, 96, 128, 160), 192: (64, 96, 128), 128: (64, 96, 128, 192, 256),
          64: (64, 128, 192, 256)}
DG_BNS8 = {256: (64, 128), 128: (128, 256)}   # 8-wave variants
DGEMM = os.environ.get("LUMEN_DGEMM", "1") != "0"
_dg_ws: dict = {}
_dg_old: list = []
_dg_plans: Optional[dict] = None


def dg_bucket(M: int) -> int:
    return next(b for b in DG_BMS if M <= b)


def decode_gemm(x: torch.Tensor, w: torch.Tensor, bm: int, bn: int, s: int, nw: int = 4,
                out: Optional[torch.Tensor] = None, flags: int = 0,
                m: Optional[int] = None) -> torch.Tensor:
    """y = x @ w^T on the decode-batch MFMA kernel with block tile (bm, bn), split-K s and nw
    (4 or 8) waves per block.  ``flags``: bit 0 rotates each tile's k loop start; bit 1 takes
    x in the k-tiled layout [K / 64, bm, 64] (``x_ktiled``) with ``m`` valid rows."""
    rows = x.shape[0] if not flags & 2 else int(m)
    y = out if out is not None else torch.empty(rows, w.shape[0], device=x.device, dtype=x.dtype)
    ws = cnt = None
    if s > 1:
        # one slab workspace + ticket counters per (device, stream): split-K slabs and tickets
        # of GEMMs on different streams never interleave (a side-stream GEMM gets its own)
        key = _dg_key(x.device)
        got = _dg_ws.get(key)
        need = -(-w.shape[0] // bn) * s * bm * bn
        if got is None or got[0].numel() < need or got[1].numel() < -(-w.shape[0] // bn):
            # generous size; a superseded pair stays alive (_dg_old): a captured decode graph
            # keeps pointing at the buffers it was captured with
            n = max(need, 1 << 24)
            if got is not None:
                _dg_old.append(got)
            got = (torch.empty(n, dtype=torch.float32, device=x.device),
                   torch.zeros(max(4096, -(-w.shape[0] // bn)), dtype=torch.int32,
                               device=x.device))
            _dg_ws[key] = got
        ws, cnt = got
    native().decode_gemm(x, w, y, ws, cnt, bm, bn, s, nw, flags)
    return y


def x_ktiled(x: torch.Tensor, bm: int = 256) -> torch.Tensor:
    """[M, K] -> [K / 64, bm, 64] (rows past M zero): the decode GEMM's k-tiled x layout."""
    M, K = x.shape
    t = torch.zeros(K // 64, bm, 64, device=x.device, dtype=x.dtype)
    t[:, :M].copy_(x.reshape(M, K // 64, 64).transpose(0, 1))
    return t


def _dg_key(device) -> tuple:
    return (str(device), torch.cuda.current_stream(device).cuda_stream)


def dg_workspace(device) -> Optional[tuple]:
    """(slab workspace, ticket counters) of the current stream on ``device`` (None before the
    first split-K call there)."""
    return _dg_ws.get(_dg_key(device))


def dg_plans() -> dict:
    """{(N, K, BM): (BN, S, waves)} from configs/kernels/decode_gemm_plans.json (measured wins only)."""
    global _dg_plans
    if _dg_plans is None:
        import json

        path = os.environ.get("LUMEN_DGEMM_PLANS", os.path.join(
            os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
            "configs", "kernels", "decode_gemm_plans.json"))
        _dg_plans = {}
        if os.path.exists(path):
            with open(path) as f:
                for e in json.load(f).get("plans", []):
                    _dg_plans[(e["N"], e["K"], e["BM"])] = (e["BN"], e["S"], e.get("NW", 4))
    return _dg_plans


def dg_plan(x: torch.Tensor, w: torch.Tensor) -> Optional[tuple]:
    if not (DGEMM and use_native(x) and x.dim() == 2 and w.dim() == 2 and 4 < x.shape[0] <= 256
            and x.dtype == w.dtype and x.dtype in (torch.bfloat16, torch.float16)
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and w.is_contiguous()
            and x.shape[1] == w.shape[1] and w.shape[1] % 64 == 0 and w.shape[0] % 4 == 0):
        return None
    bm = dg_bucket(x.shape[0])
    p = dg_plans().get((w.shape[0], w.shape[1], bm))
    return (bm,) + tuple(p) if p is not None else None


# Training-shape GEMMs run 256 x 256 macro tiles, one per CU at a time, so a GEMM with 5.375 or
# 2.69 waves of tiles on the 256-CU chip takes 6 or 3 waves (Llama-2-7B at T = 4096: gate|up
# forward 16 x 86 tiles, down input-grad 16 x 43).  ``mm_nt`` splits the output columns at the
# last whole wave and runs the remainder as its own (separately tuned) GEMM, both writing column
# views of one buffer (ldc = full width, no copies).  scripts/probes/split_gemm_probe.py measures it.
GEMM_SPLIT = os.environ.get("LUMEN_GEMM_SPLIT", "1") != "0"
SPLIT_TILE, SPLIT_CUS = 256, 256
SPLIT_MAX_TAIL = float(os.environ.get("LUMEN_GEMM_SPLIT_MAX_TAIL", "0.75"))


def split_cols(M: int, N: int) -> int:
    """Column count of the whole-wave part of an [M, N] output (0: no split).  Splits only when
    the last wave is at most ``SPLIT_MAX_TAIL`` full and the wave boundary is a column-tile
    boundary."""
    if M % SPLIT_TILE or N % 8:
        return 0
    tm, tn = M // SPLIT_TILE, -(-N // SPLIT_TILE)
    total = tm * tn
    waves, tail = divmod(total, SPLIT_CUS)
    if waves == 0 or tail == 0 or tail > SPLIT_MAX_TAIL * SPLIT_CUS or SPLIT_CUS % tm:
        return 0
    n1 = waves * (SPLIT_CUS // tm) * SPLIT_TILE
    return n1 if 0 < n1 < N else 0


_tuned: dict = {"n": -1, "sigs": frozenset()}


def _tuned_sigs() -> frozenset:
    """Problem signatures of the loaded TunableOp table (refreshed when its size changes)."""
    try:
        import torch.cuda.tunable as tn

        if not tn.is_enabled():
            return frozenset()
        res = tn.get_results()
    except Exception:  # noqa: BLE001
        return frozenset()
    if len(res) != _tuned["n"]:
        _tuned["n"], _tuned["sigs"] = len(res), frozenset(r[1] for r in res)
    return _tuned["sigs"]


def _split_plan(x: torch.Tensor, w: torch.Tensor) -> int:
    if not (GEMM_SPLIT and x.is_cuda and x.dim() == 2 and w.dim() == 2 and x.stride(1) == 1
            and w.stride(1) == 1):
        return 0
    (M, K), N = x.shape, w.shape[0]
    n1 = split_cols(M, N)
    if not n1:
        return 0
    # only where both parts have tuned solutions (untuned shapes would fall to the heuristic);
    # decided once per problem (the table is loaded before the first training GEMM)
    key = (M, N, K, w.stride(0), x.stride(0))
    hit = _plans.get(key)
    if hit is None:
        sigs = _tuned_sigs()
        lds = f"ld_{w.stride(0)}_{x.stride(0)}_{N}"
        hit = n1 if (f"tn_{n1}_{M}_{K}_{lds}" in sigs
                     and f"tn_{N - n1}_{M}_{K}_{lds}" in sigs) else 0
        _plans[key] = hit
    return hit


_plans: dict = {}


def mm_nt(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T -> [M, N] (w row-contiguous), split at the last whole wave of tiles
    on the GPU (see ``split_cols``)."""
    n1 = _split_plan(x, w)
    if not n1:
        return torch.matmul(x, w.t())
    y = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.result_type(x, w))
    torch.mm(x, w[:n1].t(), out=y[:, :n1])
    torch.mm(x, w[n1:].t(), out=y[:, n1:])
    return y


def linear_nt(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T -> [M, N]."""
    if skinny_ok(x, w):
        y = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=x.dtype)
        native().skinny_gemm(x, w, y)
        return y
    p = dg_plan(x, w)
    if p is not None:
        return decode_gemm(x, w, *p)
    # prefill / mixed steps (M = 2048-4096 tokens): the whole-wave column split where both
    # parts are tuned, as in training (profiles/r5_serve_split)
    return mm_nt(x, w)


# batch <= 4 decode, opt-in (LUMEN_SWIGLU_GEMV=1): SwiGLU formed inside the rows-per-lane weight
# stream, one launch fewer per layer.  Measured slower both ways: the row-group GEMV form 21.4 vs
# 18.5 us per call, the rows-per-lane form 3.085 vs 2.99-3.01 ms per batch-1 decode step (gpurun
# r5_35) -- every workgroup re-reads and re-activates the whole 2 x 11008 gate|up row
SWIGLU_GEMV = os.environ.get("LUMEN_SWIGLU_GEMV", "0") == "1"


def swiglu_linear_nt(gu: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """(silu(gu[:, :F]) * gu[:, F:]) @ w[N, F]^T, the MLP down projection."""
    from .activation import swiglu

    M, F = gu.shape[0], gu.shape[1] // 2
    if (SWIGLU_GEMV and 0 < M <= 4 and gu.dim() == 2 and gu.shape[1] == 2 * F
            and gu.stride(1) == 1 and gu.stride(0) % 8 == 0 and use_native(gu)
            and w.dim() == 2 and w.shape[1] == F and w.is_contiguous() and gu.dtype == w.dtype
            and gu.dtype in (torch.bfloat16, torch.float16) and w.shape[0] % 4 == 0
            and F % 8 == 0 and skinny_ok(gu[:, :F], w)):
        y = torch.empty(M, w.shape[0], device=gu.device, dtype=gu.dtype)
        native().skinny_swiglu_gemm(gu, w, y)
        return y
    return linear_nt(swiglu(gu), w)
