"""SwiGLU over a fused [gate | up] GEMM output (HIP kernel ``kernels/swiglu.hip``)."""
from __future__ import annotations

import os as _os

import torch
import torch.nn.functional as F

from ._native import native, use_native


def swiglu_ref(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        out = torch.empty(*gu.shape[:-1], gu.shape[-1] // 2, device=gu.device, dtype=gu.dtype)
        native().swiglu(False, gu, None, out)
        ctx.save_for_backward(gu)
        return out

    @staticmethod
    def backward(ctx, dact):
        (gu,) = ctx.saved_tensors
        dgu = torch.empty_like(gu)
        native().swiglu(True, gu, dact.contiguous(), dgu)
        return dgu


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if use_native(gu):
        return _SwiGLU.apply(gu)
    return swiglu_ref(gu)


class _RecomputeMLP(torch.autograd.Function):
    """down(swiglu(gate_up(y))) for frozen gate|up / down weights, keeping only ``y`` for the
    backward: the [T, 2F] gate|up output -- 5.4 H-wide rows per token, the largest activation a
    Llama layer saves -- is recomputed by one GEMM in the backward instead of being stored
    (selective activation checkpointing).  The down projection's forward is NOT re-run (full
    layer recompute does that too).  Weights are fetched through their ``weight_fn`` /
    ``weight_t_fn`` at backward time (ZeRO-3 rebinds gathered weights)."""

    @staticmethod
    def forward(ctx, y, gu_w, gu_wt, dn_w, dn_wt):
        from .gemm import mm_nt

        gu = mm_nt(y, gu_w())
        if use_native(gu):
            act = torch.empty(*gu.shape[:-1], gu.shape[-1] // 2, device=gu.device,
                              dtype=gu.dtype)
            native().swiglu(False, gu, None, act)
        else:
            act = swiglu_ref(gu)
        del gu
        out = mm_nt(act, dn_w())
        ctx.save_for_backward(y)
        ctx.fns = (gu_w, gu_wt, dn_w, dn_wt)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .gemm import mm_nt

        (y,) = ctx.saved_tensors
        gu_w, gu_wt, dn_w, dn_wt = ctx.fns
        dact = _dx(dout.contiguous(), dn_w, dn_wt)
        gu = mm_nt(y, gu_w())                     # the recompute
        if use_native(gu):
            dgu = torch.empty_like(gu)
            native().swiglu(True, gu, dact, dgu)
        else:  # the reference op's own autograd: same rounding as the unrecomputed layer
            with torch.enable_grad():
                g_ = gu.detach().requires_grad_(True)
                swiglu_ref(g_).backward(dact)
            dgu = g_.grad
        del gu, dact
        return _dx(dgu, gu_w, gu_wt), None, None, None, None


def _dx(dy, w_fn, wt_fn):
    """dX = dY @ W, as the TN GEMM against a cached W^T when the layer keeps one."""
    from .gemm import mm_nt

    wt = wt_fn() if wt_fn is not None else None
    return mm_nt(dy, wt) if wt is not None else torch.matmul(dy, w_fn())


# LUMEN_MLP_OVERLAP (opt-in): the frozen MLP's wave-quantization tails run on a side stream
# beside the activation of the columns already produced (0 = off; 1 = the tail GEMM starts after
# the whole-wave part, beside the SwiGLU of that part; 2 = the tail is issued at once and competes
# with the whole-wave part for CUs).  Measured slower (profiles/r5_mlp_overlap): 93.3 / 91.2 vs
# 90.7 ms per step -- beside the SwiGLU's thousands of small workgroups the 1536-column tail GEMM
# took 102 instead of 52 us, and the SwiGLU passes slowed too.
MLP_OVERLAP = int(_os.environ.get("LUMEN_MLP_OVERLAP", "0"))
_side: dict = {}


def _side_stream(dev) -> "torch.cuda.Stream":
    s = _side.get(dev)
    if s is None:
        s = _side[dev] = torch.cuda.Stream(device=dev)
    return s


def _split_gemm_act(x, w, n1, out, act_fn, c_ready, c_end):
    """out = x @ w^T split at column n1: the whole-wave part [0, n1) on the current stream, the
    tail [n1, N) on a side stream; ``act_fn(c0, c1)`` runs the activation of columns [0,
    c_ready) beside the tail, then [c_ready, c_end) after the join."""
    cur = torch.cuda.current_stream(x.device)
    side = _side_stream(x.device)
    if MLP_OVERLAP == 2:
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            torch.mm(x, w[n1:].t(), out=out[:, n1:])
        torch.mm(x, w[:n1].t(), out=out[:, :n1])
    else:
        torch.mm(x, w[:n1].t(), out=out[:, :n1])
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            torch.mm(x, w[n1:].t(), out=out[:, n1:])
    act_fn(0, c_ready)
    cur.wait_stream(side)
    act_fn(c_ready, c_end)


class _OverlapMLP(torch.autograd.Function):
    """down(swiglu(gate_up(y))) for frozen, adapter-free gate|up / down weights on the GPU, with
    each wave-quantized GEMM's tail hidden under the memory-bound SwiGLU pass.

    * Forward: gate|up [T, 2F] splits at its last whole wave of 256 x 256 tiles (Llama-2-7B at
      T = 4096: columns 20480 + 1536; the tail runs at ~1 PF/s on a third of the CUs).  The
      SwiGLU of activation columns [0, n1 - F) -- all their gate and up inputs are in the whole-
      wave part -- runs while the tail computes on a side stream; the rest follows the join.
    * Backward: dact = dout @ W_down splits the same way (11008 = 8192 + 2816 at T = 4096), and
      the SwiGLU backward of columns [0, 8192) runs beside its tail.
    Saves the gate|up output (as the unfused path does); same kernels, same rounding."""

    @staticmethod
    def forward(ctx, y, gu_w, gu_wt, dn_w, dn_wt, n1):
        from .gemm import mm_nt

        w = gu_w()
        T, F = y.shape[0], w.shape[0] // 2
        gu = torch.empty(T, 2 * F, device=y.device, dtype=y.dtype)
        act = torch.empty(T, F, device=y.device, dtype=y.dtype)
        _split_gemm_act(y, w, n1, gu, lambda c0, c1: native().swiglu(False, gu, None, act, c0, c1),
                        n1 - F, F)
        out = mm_nt(act, dn_w())
        ctx.save_for_backward(gu)
        ctx.fns = (gu_w, gu_wt, dn_w, dn_wt)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .gemm import _split_plan

        (gu,) = ctx.saved_tensors
        gu_w, gu_wt, dn_w, dn_wt = ctx.fns
        dout = dout.contiguous()
        F = gu.shape[1] // 2
        wt = dn_wt() if dn_wt is not None else None
        n1 = _split_plan(dout, wt) if wt is not None else 0
        dgu = torch.empty_like(gu)
        if n1:
            dact = torch.empty(gu.shape[0], F, device=gu.device, dtype=gu.dtype)
            _split_gemm_act(dout, wt, n1, dact,
                            lambda c0, c1: native().swiglu(True, gu, dact, dgu, c0, c1), n1, F)
        else:
            dact = _dx(dout, dn_w, dn_wt)
            native().swiglu(True, gu, dact, dgu)
        del dact
        return _dx(dgu, gu_w, gu_wt), None, None, None, None, None


def overlap_mlp_plan(y: torch.Tensor, gate_up, down) -> int:
    """The gate|up split column for ``_OverlapMLP`` (0: not applicable): GPU, native kernels,
    frozen adapter-free weights, and a tuned whole-wave split whose first part holds every gate
    column."""
    if not (MLP_OVERLAP and y.is_cuda and y.dim() == 2 and use_native(y)
            and gate_up.bias is None and down.bias is None):
        return 0
    from .gemm import _split_plan

    w = gate_up.weight_fn()
    n1 = _split_plan(y, w) if w.is_contiguous() else 0
    F = w.shape[0] // 2
    return n1 if F < n1 and (n1 - F) % 8 == 0 else 0


def overlap_mlp(y: torch.Tensor, gate_up, down, n1: int) -> torch.Tensor:
    return _OverlapMLP.apply(y.contiguous(), gate_up.weight_fn, gate_up._wt_fn(),
                             down.weight_fn, down._wt_fn(), n1)


# LUMEN_FUSED_MLP: the frozen MLP's gate|up GEMM with the SwiGLU in its epilogue, and the
# down projection's input-gradient GEMM with the SwiGLU backward in its epilogue (hand-written
# gfx950 GEMM, kernels/mlp_gemm.hip; VERDICT r5 Next #1).  1 = both, fwd / bwd = one of them,
# 0 = off (library GEMMs + the separate SwiGLU passes).
FUSED_MLP = _os.environ.get("LUMEN_FUSED_MLP", "0")


def _mlp_gemm_ok(x: torch.Tensor, w: torch.Tensor, col_mult: int) -> bool:
    return (x.dim() == 2 and w.dim() == 2 and x.stride(1) == 1 and w.stride(1) == 1
            and x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0 and x.shape[1] == w.shape[1]
            and x.shape[1] % 64 == 0 and x.dtype == w.dtype
            and x.dtype in (torch.bfloat16, torch.float16) and w.shape[0] % col_mult == 0
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


class _FusedMLP(torch.autograd.Function):
    """down(swiglu(gate_up(y))) for frozen, adapter-free weights with the activation inside the
    GEMM epilogues (kernels/mlp_gemm.hip):

    * forward: ONE launch writes gu (saved for the backward) and act = silu(g) * u; the down
      projection is the library GEMM;
    * backward: dact = dout @ Wd (against the cached Wd^T) in ONE launch whose epilogue reads
      g / u and writes dg | du -- dact never reaches HBM; dX = dgu @ W_gu is the library GEMM.
    Each half falls back to the separate passes where the kernel does not take the layout."""

    @staticmethod
    def forward(ctx, y, gu_w, gu_wt, dn_w, dn_wt, mode):
        from .gemm import mm_nt

        w = gu_w()
        T, F = y.shape[0], w.shape[0] // 2
        if mode in ("1", "fwd") and _mlp_gemm_ok(y, w, 256):
            gu = torch.empty(T, 2 * F, device=y.device, dtype=y.dtype)
            act = torch.empty(T, F, device=y.device, dtype=y.dtype)
            from .mlp_gemm import mlp_gemm

            mlp_gemm(1, y, w, gu, act)
        else:
            gu = mm_nt(y, w)
            act = torch.empty(T, F, device=y.device, dtype=y.dtype)
            native().swiglu(False, gu, None, act, 0, -1)
        out = mm_nt(act, dn_w())
        ctx.save_for_backward(gu)
        ctx.fns = (gu_w, gu_wt, dn_w, dn_wt)
        ctx.mode = mode
        return out

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        gu_w, gu_wt, dn_w, dn_wt = ctx.fns
        dout = dout.contiguous()
        F = gu.shape[1] // 2
        wdt = dn_wt() if dn_wt is not None else None   # Wd^T [F, H]
        dgu = torch.empty_like(gu)
        if (ctx.mode in ("1", "bwd") and wdt is not None and F % 256 == 0
                and _mlp_gemm_ok(dout, wdt, 256)):
            from .mlp_gemm import mlp_gemm

            mlp_gemm(2, dout, wdt, dgu, None, gu)
        else:
            dact = _dx(dout, dn_w, dn_wt)
            native().swiglu(True, gu, dact, dgu, 0, -1)
            del dact
        return _dx(dgu, gu_w, gu_wt), None, None, None, None, None


def fused_mlp_ok(y: torch.Tensor, gate_up, down) -> bool:
    """The fused-epilogue MLP applies: LUMEN_FUSED_MLP on, GPU native kernels, 16-bit 2-D
    activations, frozen adapter-free bias-free weights, F a multiple of 256."""
    if FUSED_MLP in ("0", "") or not (y.is_cuda and y.dim() == 2 and use_native(y)):
        return False
    if gate_up.bias is not None or down.bias is not None:
        return False
    w = gate_up.weight
    return (w.dim() == 2 and w.shape[0] % 512 == 0 and y.dtype in (torch.bfloat16, torch.float16)
            and hasattr(native(), "mlp_gemm"))


def fused_mlp(y: torch.Tensor, gate_up, down) -> torch.Tensor:
    return _FusedMLP.apply(y.contiguous(), gate_up.weight_fn, gate_up._wt_fn(), down.weight_fn,
                           down._wt_fn(), FUSED_MLP)


def recompute_mlp(y: torch.Tensor, gate_up, down) -> torch.Tensor:
    """Selective-recompute MLP over two frozen, adapter-free ``Linear`` modules (see
    ``_RecomputeMLP``)."""
    return _RecomputeMLP.apply(y.contiguous(), gate_up.weight_fn, gate_up._wt_fn(),
                               down.weight_fn, down._wt_fn())
