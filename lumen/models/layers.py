"""Building blocks shared by the model families: (LoRA-capable) fused linear layers, norms.

``Linear`` owns a (usually frozen) base weight [out, in] and an optional LoRA adapter covering
one or more output segments (q|k|v fused, gate|up fused).  The weight is always read through
``self.weight_fn`` at forward AND backward time, so ZeRO-3's parameter coordinator can release a
gathered weight after the forward and re-gather it before the backward without autograd pinning
the full tensor.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from ..ops import lora as lora_ops
from ..ops.lora import lora_linear, linear
from ..ops.transpose import transpose_2d
from ..ops.norm import rms_norm


class LoRAAdapter(nn.Module):
    """Stacked adapter for the adapted output segments of a (fused) linear layer.

    lora_A: [n_seg * r, in]   rows r_off..r_off+r = segment's PEFT ``lora_A.weight`` [r, in]
    lora_B: [sum(out_i), r]   rows b_off..b_off+out_i = segment's PEFT ``lora_B.weight`` [out_i, r]
    ``segs`` = (n_off, n_len, r_off, b_off) with n_off the absolute output column of the segment.
    """

    def __init__(self, in_features: int, seg_offsets: Sequence[int], seg_sizes: Sequence[int],
                 names: Sequence[str], r: int, alpha: float, dropout: float, device=None):
        super().__init__()
        self.r, self.alpha, self.dropout = r, alpha, dropout
        self.scale = alpha / r
        self.names = list(names)
        self.seg_sizes = list(seg_sizes)
        self.in_features = in_features
        n = len(seg_sizes)
        self.lora_A = nn.Parameter(torch.empty(n * r, in_features, dtype=torch.float32, device=device))
        self.lora_B = nn.Parameter(torch.zeros(sum(seg_sizes), r, dtype=torch.float32, device=device))
        self.segs: List[Tuple[int, int, int, int]] = []
        b = 0
        for i, (o, sz) in enumerate(zip(seg_offsets, seg_sizes)):
            self.segs.append((o, sz, i * r, b))
            b += sz
        self.reset_parameters()

    def reset_parameters(self):
        # PEFT: kaiming_uniform_(A, a=sqrt(5)) -> U(-1/sqrt(in), 1/sqrt(in)); B = 0
        bound = 1.0 / math.sqrt(self.in_features)
        with torch.no_grad():
            self.lora_A.uniform_(-bound, bound)
            self.lora_B.zero_()

    def segment(self, name: str):
        """(A_i, B_i) views for PEFT save/load."""
        i = self.names.index(name)
        n_off, n_len, r_off, b_off = self.segs[i]
        return self.lora_A[r_off:r_off + self.r], self.lora_B[b_off:b_off + n_len]


class Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = False, dtype=None,
                 device=None, seg_sizes: Optional[Sequence[int]] = None,
                 seg_names: Optional[Sequence[str]] = None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype, device=device),
                                   requires_grad=False)
        self.bias = (nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device),
                                  requires_grad=False) if bias else None)
        self.seg_sizes = list(seg_sizes) if seg_sizes else [out_features]
        self.seg_names = list(seg_names) if seg_names else ["proj"]
        self.lora: Optional[LoRAAdapter] = None
        self.lora_enabled = True
        self.transpose_bwd = False      # keep W^T for a K-contiguous (TN) input-gradient GEMM
        self.transpose_gathered = False  # ... also for ZeRO-3-gathered weights (per step)
        self._wt: Optional[torch.Tensor] = None
        self._wt_key = None
        self._wext: Optional[torch.Tensor] = None  # [W | s B_bd | 0] (LoRA fold), see fold_weight
        self._wext_key = None
        self._tail_key = None

    def weight_fn(self) -> torch.Tensor:
        return self.weight

    def weight_t_fn(self) -> Optional[torch.Tensor]:
        """Contiguous W^T [in, out] for the backward dX = dY @ W, or None.

        hipBLASLt runs dY[T,N] @ W[N,K] (reduction over W's row index) markedly slower than the
        TN form dY @ (W^T)^T with both operands K-contiguous (lumen/bench/gemm_bench.py), so
        frozen persistent weights keep a transposed copy (288 GB HBM affords it).  ZeRO-3
        gathered weights change storage every step: they are transposed on the fly, and only
        where the GEMM saving beats the transpose's HBM traffic (``transpose_gathered``)."""
        W = self.weight
        if not self.transpose_bwd or W.requires_grad:
            return None
        if getattr(W, "_lumen_gathered", False):
            wt = getattr(W, "_lumen_wt", None)  # transposed by the ZeRO-3 coordinator off-path
            if wt is not None:
                return wt
            return transpose_2d(W.detach()) if self.transpose_gathered else None
        key = (W.data_ptr(), tuple(W.shape), W.dtype)
        if self._wt is None or self._wt_key != key:
            with torch.no_grad():
                self._wt = transpose_2d(W.detach())
            self._wt_key = key
        return self._wt

    def invalidate_weight_cache(self):
        self._wt, self._wt_key = None, None
        self._wext, self._wext_key, self._tail_key = None, None, None

    # ---- LoRA fold: forward UP folded into the frozen-weight GEMM as 64 extra K columns --------
    def fold_ext(self, static: bool = False) -> int:
        """Extra operand columns this linear's producer should leave after x (0 = no fold).
        ``static``: eligibility of the layer itself (the ZeRO-3 layout asks before the weight
        is partitioned); otherwise also of the weight as currently bound."""
        lo, W = self.lora, self.weight
        if (not lora_ops.FOLD or lo is None or not self.lora_enabled or W.requires_grad
                or not W.is_cuda or W.dtype not in (torch.bfloat16, torch.float16)
                or not lora_ops.use_native(W)):
            return 0
        if not static:
            if W.dim() != 2 or W.numel() == 0:
                return 0
            # gathered ZeRO-3 weights fold only when the partitioned layout reserved the tail
            if getattr(W, "_lumen_gathered", False) and (
                    getattr(W, "_lumen_fold_kp", 0) != lora_ops.FOLD_KP
                    or W.stride(0) != self.in_features + lora_ops.FOLD_KP):
                return 0
        K = self.in_features
        R = lo.lora_A.shape[0]
        if (lo.r not in (16, 32, 64) or R > lora_ops.FOLD_KP or K % 8
                or any(sg[0] % 8 or sg[1] % 8 or sg[2] % 8 for sg in lo.segs)
                or lo.lora_A.dtype != torch.float32 or not lo.lora_B.is_contiguous()):
            return 0
        return lora_ops.FOLD_KP

    def fold_weight(self) -> Optional[torch.Tensor]:
        """[N, K + 64] bf16/fp16 = [W | s B_bd | 0]: W copied when the weight changes, the tail
        (scale x lora_B, block-diagonal over segments) refreshed when lora_B changes (the
        engine's optimizer publish bumps its version counter, FlatTrainable.mark_updated; after a
        synchronous publish FoldTails has usually refreshed every tail in one launch already)."""
        if not self.fold_ext():
            return None
        wext, tkey = self._fold_target()
        if self._tail_key != tkey:
            self._fill_tail(wext)
            self._tail_key = tkey
        return wext

    def _fold_target(self):
        """(extended weight, tail key) of this linear's fold.  The weight itself when it lives
        in [N, K + KP] rows (ZeRO-3 layout: the tail is rewritten in place -- a fresh gather
        clears the key, ParamCoordinator -> invalidate_fold_tail; a resident unit keeps it until
        lora_B's version moves), else a cached [W | 0] copy rebuilt when W changes."""
        lo, W = self.lora, self.weight
        K, KP = self.in_features, lora_ops.FOLD_KP
        if W.stride(0) == K + KP and W.stride(1) == 1:
            wext = W.as_strided((W.shape[0], K + KP), (K + KP, 1))
            return wext, (W.data_ptr(), lo.lora_B.data_ptr(), lo.lora_B._version, lo.scale)
        key = (W.data_ptr(), W._version, tuple(W.shape), W.dtype)
        if self._wext is None or self._wext_key != key:
            with torch.no_grad():
                self._wext = torch.zeros(W.shape[0], K + KP, dtype=W.dtype, device=W.device)
                self._wext[:, :K].copy_(W)
            self._wext_key = key
            self._tail_key = None
        B = lo.lora_B
        return self._wext, (B.data_ptr(), B._version, lo.scale)

    def _fill_tail(self, wext: torch.Tensor) -> None:
        from ..ops._native import native

        lo = self.lora
        native().lora3_w_tail(wext, self.in_features, lo.lora_B.detach(), lo.r,
                              [(n_off, b_off, n_len, r_off)
                               for (n_off, n_len, r_off, b_off) in lo.segs], lo.scale)

    def tail_desc(self, wext: torch.Tensor) -> Optional[list]:
        """The 24-int64 row of FoldTails' batched launch for this linear, or None when its
        layout is not one the batched kernel takes (the per-linear fill then runs)."""
        import struct

        lo, K = self.lora, self.in_features
        B = lo.lora_B
        if (lo.r % 8 or K % 8 or wext.stride(0) % 8 or wext.stride(1) != 1
                or not B.is_contiguous() or B.dtype != torch.float32 or len(lo.segs) > 4
                or any(r_off % 8 for (_, _, r_off, _) in lo.segs)):
            return None
        d = [wext.data_ptr(), wext.stride(0), B.data_ptr(), K, lo.r, len(lo.segs),
             struct.unpack("<I", struct.pack("<f", float(lo.scale)))[0], 0]
        segs = list(lo.segs) + [(0, 0, 0, 0)] * (4 - len(lo.segs))
        d += [sg[0] for sg in segs] + [sg[1] for sg in segs] + [sg[2] for sg in segs] + [
            sg[3] for sg in segs]
        return d

    def invalidate_fold_tail(self) -> None:
        """ZeRO-3: the unit was just gathered, so the tail columns of its [N, K + KP] rows hold
        the shard's padding; the next ``fold_weight()`` writes s * lora_B there."""
        self._tail_key = None

    def seg_offset(self, name: str) -> Tuple[int, int]:
        i = self.seg_names.index(name)
        return sum(self.seg_sizes[:i]), self.seg_sizes[i]

    def add_lora(self, names: Sequence[str], r: int, alpha: float, dropout: float):
        names = sorted(names, key=self.seg_names.index)
        offs = [self.seg_offset(n)[0] for n in names]
        sizes = [self.seg_offset(n)[1] for n in names]
        self.lora = LoRAAdapter(self.in_features, offs, sizes, names, r, alpha, dropout,
                                device=self.weight.device)
        return self.lora

    @property
    def has_active_lora(self) -> bool:
        return self.lora is not None and self.lora_enabled

    def forward(self, x: torch.Tensor, rope=None) -> torch.Tensor:
        """``rope`` (only with an active adapter on the GPU path): see ``lora_linear``."""
        lo = self.lora
        if lo is not None and self.lora_enabled:
            p = lo.dropout if self.training else 0.0
            # seed drawn from torch's global CPU RNG: activation checkpointing restores that state
            # before recomputing, so the recomputed forward regenerates the same dropout mask
            seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
            fold = (self.fold_weight() if x.dim() == 2
                    and lora_ops.fold_operand(x, self.in_features) is not None else None)
            return lora_linear(x, self.weight_fn, self.bias, lo.lora_A, lo.lora_B, lo.segs, lo.r,
                               lo.scale, p, seed, self.weight, self._wt_fn(), rope, fold)
        if rope is not None:
            raise ValueError("fused RoPE needs an active LoRA adapter on this linear")
        return linear(x, self.weight_fn, self.bias, self.weight, self._wt_fn())

    def _wt_fn(self):
        return self.weight_t_fn if (self.transpose_bwd and torch.is_grad_enabled()) else None

    @torch.no_grad()
    def merge_lora(self):
        """W += scale * B A for every adapted segment (serving: merge-on-load)."""
        lo = self.lora
        if lo is None:
            return
        W = self.weight
        for (n_off, n_len, r_off, b_off) in lo.segs:
            A = lo.lora_A[r_off:r_off + lo.r].float()
            B = lo.lora_B[b_off:b_off + n_len].float()
            W[n_off:n_off + n_len] = (W[n_off:n_off + n_len].float() + lo.scale * (B @ A)).to(W.dtype)
        self.lora = None
        self.invalidate_weight_cache()


GATHERED_TN = ("q_proj", "down_proj", "fc2")


def _gathered_tn() -> tuple:
    """Linears whose ZeRO-3-gathered weights get a per-step W^T (env ``LUMEN_GATHERED_TN``:
    comma list of first-segment names, overriding ``GATHERED_TN``)."""
    import os

    e = os.environ.get("LUMEN_GATHERED_TN")
    return GATHERED_TN if e is None else tuple(x for x in e.split(",") if x)


def configure_backward_layout(model: nn.Module, policy=None) -> int:
    """Enable the transposed-weight (TN) input-gradient GEMM on the linears whose first segment
    name is in ``policy`` (env ``LUMEN_BWD_WT``: comma list, ``all`` or ``none``; default
    ``all``: in-situ on MI355X the TN form won for every Llama-2-7B projection -- step time
    104.6 ms vs 110.0 ms with none, profiles/r01_tuned).  Returns the count enabled."""
    import os

    if policy is None:
        policy = os.environ.get("LUMEN_BWD_WT", "all")
    if isinstance(policy, str):
        policy = policy.strip()
        names = None if policy == "all" else set() if policy in ("", "none") else set(policy.split(","))
    else:
        names = set(policy)
    budget = _transpose_budget(model)
    gathered_tn = _gathered_tn()
    n = 0
    for name, m in model.named_modules():
        if isinstance(m, Linear):
            # the LM head too (LUMEN_LMHEAD_WT=0: not): its dH = dlogits @ W measured 874 -> 778 us
            # as the TN GEMM against W^T (Llama-2-7B, 8 x 512 tokens, gpurun r5_55)
            head_ok = not name.endswith("lm_head") or os.environ.get("LUMEN_LMHEAD_WT", "1") != "0"
            on = head_ok and (names is None or m.seg_names[0] in names)
            gathered = getattr(m.weight, "_lumen_gathered", False)
            if on and not gathered:  # persistent copies must fit the HBM budget
                need = m.weight.numel() * m.weight.element_size()
                on = need <= budget
                budget -= need if on else 0
            m.transpose_bwd = on
            # per-step transposes of gathered weights pay off where the NN GEMM is slowest
            # relative to the transpose's traffic (q|k|v: 299 -> 188 us, down: 277 -> 200 us)
            m.transpose_gathered = on and m.seg_names[0] in gathered_tn
            m.invalidate_weight_cache()
            n += int(on)
    return n


def _transpose_budget(model: nn.Module) -> float:
    """Bytes of HBM the persistent W^T copies may take: free memory minus a reserve for
    activations (max(48 GiB, 25% of the device)); unlimited off-GPU."""
    import os

    dev = next((p.device for p in model.parameters() if p.device.type == "cuda"), None)
    if dev is None:
        return float("inf")
    free, total = torch.cuda.mem_get_info(dev)
    # blocks the caching allocator holds but no tensor uses (e.g. init temporaries) are free
    # for the W^T copies too (mem_get_info counts them as used)
    free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    from ..parallel.memory_plan import activation_reserve

    return max(0.0, free - activation_reserve(total, "LUMEN_BWD_WT_RESERVE_GB"))


def invalidate_weight_caches(model: nn.Module) -> None:
    for m in model.modules():
        if isinstance(m, Linear):
            m.invalidate_weight_cache()


class RMSNorm(nn.Module):
    def __init__(self, hidden: int, eps: float, dtype=None, device=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden, dtype=dtype, device=device), requires_grad=False)

    def forward(self, x, residual=None, ext: int = 0):
        """``ext`` > 0: y is written into the first H columns of a [rows, H + ext] buffer and
        returned as that view (the operand of a K-extended LoRA GEMM, ``Linear.fold_ext``)."""
        return rms_norm(x, self.weight, self.eps, residual, ext)


class FoldTails:
    """Refresh every folded linear's [s B] tail in ONE launch (``kernels/lora_v3.hip``
    w_tail_batch_kernel) right after a synchronous optimizer publish, instead of one small launch
    per linear inside the next forward (64 launches, ~0.3 ms per Llama-2-7B step).  Linears it
    cannot cover (unbound ZeRO-3 release units, odd layouts) keep the lazy per-linear fill."""

    def __init__(self, model: nn.Module):
        self.lins = [m for m in model.modules() if isinstance(m, Linear) and m.lora is not None]
        self._desc: Optional[torch.Tensor] = None
        self._sig = None
        self._meta = (0, 0)

    def refresh(self) -> int:
        """Returns the number of tails written (0: nothing to do here)."""
        from ..ops._native import native

        C = native()
        lins = [m for m in self.lins if m.weight.is_cuda and m.fold_ext()]
        if not lins or C is None or not hasattr(C, "lora3_w_tail_batch"):
            return 0
        targets = [m._fold_target() for m in lins]
        rows = [m.tail_desc(w) for m, (w, _) in zip(lins, targets)]
        keep = [i for i, r in enumerate(rows) if r is not None]
        dts = {targets[i][0].dtype for i in keep}
        if not keep or len(dts) != 1:
            return 0
        sig = tuple(tuple(rows[i]) for i in keep)
        if sig != self._sig:
            dt = dts.pop()
            code = {torch.bfloat16: 2, torch.float16: 1}.get(dt)
            if code is None:
                return 0
            self._desc = torch.tensor([rows[i] for i in keep], dtype=torch.int64).pin_memory().to(
                lins[0].weight.device, non_blocking=True)
            max_chunks = max(rows[i][12 + s] * (rows[i][4] // 8) for i in keep for s in range(4))
            self._meta = (code, max_chunks)
            self._sig = sig
        C.lora3_w_tail_batch(self._desc, *self._meta)
        for i in keep:
            lins[i]._tail_key = targets[i][1]
        return len(keep)
