"""LoRA linear: frozen base GEMM (hipBLASLt) + adapter GEMMs (HIP MFMA kernel ``kernels/lora.hip``).

Reference behaviour: PEFT LoraLayer (reference training/train_baseline.py:131-141): for each
adapted projection  y = x W^T + b + (alpha / r) * B(A(dropout(x))).  Here several projections
that share the input (q|k|v, or gate|up) are ONE base GEMM over a fused weight and ONE adapter
"A" GEMM over the stacked A matrices; each output segment then gets its own B product added in
place.  Adapter weights are f32 (PEFT keeps adapters in f32); the adapter math is f32-exact.

Segments: list of ``(n_off, n_len, r_off, b_off)``: output columns [n_off, n_off+n_len) use
adapter rows A[r_off:r_off+r] and B[b_off:b_off+n_len, :] (B stores only adapted segments).

Dropout uses a counter-based hash of (seed, token*K + feature) so the backward regenerates the
forward's mask instead of storing a [T, K] tensor; ``dropout_mask_ref`` is the same hash in
torch (bit-identical), used by the CPU path and the tests.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from ._native import DTYPE_CODE, native, use_native
from .gemm import mm_nt

Seg = Tuple[int, int, int, int]

_M32 = 0xFFFFFFFF


def _lowbias32(x):
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def seed32(seed: int) -> int:
    """The 32-bit seed the kernels use (same folding as the native launcher)."""
    seed &= 0x7FFFFFFFFFFFFFFF
    return (seed ^ (seed >> 32)) & _M32


def rng_u32_ref(seed: int, idx: torch.Tensor) -> torch.Tensor:
    s = seed32(seed)
    h = ((idx & _M32) * 0x9E3779B1 + (idx >> 32) * 0x85EBCA77 + s) & _M32
    return _lowbias32(h)


def drop_threshold(p: float) -> int:
    """16-bit drop threshold: element dropped when its 16-bit hash slice < p * 65536."""
    return min(int(round(p * 65536.0)), 0xFFFF) if p > 0 else 0


def dropout_mask_ref(seed: int, T: int, K: int, p: float, device=None) -> torch.Tensor:
    """Keep-mask [T, K] (bool) identical to the kernels': one 32-bit hash per element pair
    (index >> 1), low 16 bits for the even element, high 16 bits for the odd one."""
    idx = torch.arange(T * K, dtype=torch.int64, device=device).view(T, K)
    h = rng_u32_ref(seed, idx >> 1)
    return ((h >> ((idx & 1) * 16)) & 0xFFFF) >= drop_threshold(p)


def _apply_dropout_ref(x, p, seed):
    if p <= 0:
        return x
    keep = dropout_mask_ref(seed, x.shape[0], x.shape[1], p, x.device)
    return torch.where(keep, x.float() / (1.0 - p), torch.zeros((), device=x.device)).to(x.dtype)


# ----------------------------------------------------------------------------------------------
# native launches
# ----------------------------------------------------------------------------------------------

def _ksplit(M, N, K, bn, nseg=1, target_blocks=1024, max_atomic=2_000_000, min_k=128):
    tiles = math.ceil(M / 64) * math.ceil(N / bn) * nseg
    ks = max(1, math.ceil(target_blocks / max(tiles, 1)))
    ks = min(ks, max(1, math.ceil(K / min_k)), max(1, max_atomic // max(M * N * nseg, 1)))
    return int(ks)


def _bn(N):
    return 16 if N <= 16 else 64


def _lora_gemm(act, mode, X, W, Cm, ldx, ldw, cs_m, cs_n, alpha, segs6, ksplit, seed=0,
               p=0.0, drop_ld=0):
    bn = _bn(max(s[4] for s in segs6))
    thresh = drop_threshold(p)
    dscale = 1.0 / (1.0 - p) if p > 0 else 1.0
    native().lora_gemm(act, mode, bn, X, W, Cm, ldx, ldw, cs_m, cs_n, float(alpha), int(ksplit),
                       int(seed) & 0x7FFFFFFFFFFFFFFF, thresh, dscale, drop_ld,
                       [list(map(int, s)) for s in segs6])


import os as _os

USE_V2 = _os.environ.get("LUMEN_LORA_V2", "1") != "0"


def _v2_ok(r: int, R: int, *mats) -> bool:
    """The 16-bit-MFMA kernels (kernels/lora_v2.hip) take ranks that are multiples of 16 up to
    64 stacked rows and 8-element aligned rows; anything else uses the f32-MFMA kernel."""
    return (USE_V2 and r % 16 == 0 and R % 16 == 0 and R <= 64
            and all(m.stride(0) % 8 == 0 and m.stride(1) == 1 for m in mats))


SPLIT_TARGET = int(_os.environ.get("LUMEN_LORA_SPLIT_TARGET", "512"))  # blocks per launch


def _split(blocks_per_split: int, reduce_len: int, chunk: int, target: int = 0) -> int:
    s = max(1, math.ceil((target or SPLIT_TARGET) / max(blocks_per_split, 1)))
    return int(max(1, min(s, reduce_len // chunk)))


def _lora2(kind, flag, big, small, out, cs0, cs1, alpha, T, J, split, segs4, seed=0, p=0.0,
           drop_ld=0, rope=None):
    dt = DTYPE_CODE[out.dtype if kind == 2 else big.dtype]
    native().lora2(dt, kind, flag, big, big.stride(0), small, small.stride(0), out, cs0, cs1, float(alpha), T, J, int(split),
                   int(seed) & 0x7FFFFFFFFFFFFFFF, drop_threshold(p),
                   1.0 / (1.0 - p) if p > 0 else 1.0, drop_ld, 0,
                   [list(map(int, s)) for s in segs4],
                   *(rope if rope is not None else (None, None, None, 0)))


class ZeroArena:
    """Pre-zeroed f32 scratch for the adapter kernels' atomic accumulators (Z, dZ).

    Every adapted linear needs two zero-initialised [T, R] buffers per micro-step; handing out
    slices of one buffer that is zeroed once per forward (``reset``) replaces ~128 fill kernels
    per Llama-2-7B step with one.  A cycle that outgrows the buffer falls back to torch.zeros
    and the next ``reset`` reallocates to the measured demand.  Slices stay valid until the next
    ``reset``, i.e. through the backward of the same micro-step."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.off = 0      # bytes handed out of buf (in elements)
        self.used = 0     # demand of the current cycle, including fallbacks

    def reset(self, device) -> None:
        if self.buf is None or self.buf.device != device or self.buf.numel() < self.used:
            self.buf = (torch.zeros(self.used, device=device, dtype=torch.float32)
                        if self.used else None)
        elif self.off:
            self.buf[:self.off].zero_()
        self.off = 0
        self.used = 0

    def zeros(self, *shape, device) -> torch.Tensor:
        n = math.prod(shape)
        n_al = (n + 63) // 64 * 64
        self.used += n_al
        if self.buf is not None and self.buf.device == device and self.off + n_al <= self.buf.numel():
            t = self.buf[self.off:self.off + n].view(*shape)
            self.off += n_al
            return t
        return torch.zeros(*shape, device=device, dtype=torch.float32)


ARENA = ZeroArena()
USE_ARENA = _os.environ.get("LUMEN_LORA_ARENA", "1") != "0"
_IN_BACKWARD = [False]


def arena_reset(device) -> None:
    """Start of a training forward (called by the model); no-op unless enabled on a GPU."""
    if USE_ARENA and device.type == "cuda":
        ARENA.reset(device)


def _zeros(*shape, device, train: bool = False):
    if USE_ARENA and device.type == "cuda" and (train or _IN_BACKWARD[0]):
        return ARENA.zeros(*shape, device=device)
    return torch.zeros(*shape, device=device, dtype=torch.float32)


USE_V3 = _os.environ.get("LUMEN_LORA_V3", "1") != "0"
DY_TW = int(_os.environ.get("LUMEN_LORA_DY_TW", "0"))  # dY rows per block of lora3_dy (0 = auto)
DXA_TW = int(_os.environ.get("LUMEN_LORA_DXA_TW", "0"))  # x rows per block of lora3_dxa (0 = auto)
# deterministic mode: the forward Z, the dY pass's dZ / dB and the x pass's dA sums as second
# whole-chip launches (1) or inside the kernels by the last-arriving workgroups (0)
DET_SPLIT = _os.environ.get("LUMEN_DET_SPLIT", "1") != "0"
# per-call A/B (scripts/probes/lora_kernels.py, us): the v3 UP write-back was on par with v2
# without RoPE (o_proj 15.0 vs 14.3) and slower with it (q|k|v 55.7 vs 45.6), so v2 is the
# forward UP; v3's DOWN (17.3 vs 21.9), fused dY pass (32.5 vs 53.3) and dx update win.  A
# partial-sum + reduce variant of the dY pass (instead of f32 atomics) measured neutral and was
# removed (profiles/r2_lora).
# fused x-side backward (dA + dx in one pass over the activation rows, lora3_dxa)
DXA = _os.environ.get("LUMEN_LORA_DXA", "1") != "0"
# flash-attention delta hand-off: when this linear's input is a flash-attention output O (it
# carries ``_lumen_delta_slot``), the fused dA + dx kernel also writes delta = rowsum(dO * O) per
# head for the attention backward, which then skips its own delta pass (LUMEN_FA_DELTA_HANDOFF=0:
# off).  The slot of the linear whose backward is running:
DELTA_HANDOFF = _os.environ.get("LUMEN_FA_DELTA_HANDOFF", "1") != "0"
_DELTA_SLOT = [None]


# Deterministic adapter reductions (VERDICT r5 Next #4; kernels/det.h): the v3 down / dY / dA
# passes sum their cross-workgroup partials through write-through slabs and a last-arriver fixed
# order instead of f32 atomics, so two runs with the same seed give bit-identical adapter
# gradients.  Opt-in (LUMEN_LORA_DETERMINISTIC=1): it costs step time (profiles/r6_det).
DETERMINISTIC = _os.environ.get("LUMEN_LORA_DETERMINISTIC", "0") == "1"
_det: dict = {}


def _det_ws(dev, nfloat: int, ncnt: int):
    """(f32 slab workspace, zeroed int32 ticket counters) of the current stream on ``dev``;
    counters are left zeroed by every launch, so they are shared by the kernels in stream order."""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    got = _det.get(key)
    if got is None or got[0].numel() < nfloat or got[1].numel() < ncnt:
        nf = max(nfloat, got[0].numel() if got is not None else 0, 1 << 20)
        nc = max(ncnt, got[1].numel() if got is not None else 0, 4096)
        got = (torch.empty(nf, dtype=torch.float32, device=dev),
               torch.zeros(nc, dtype=torch.int32, device=dev))
        _det[key] = got
    return got


def _v3_ok(r: int, R: int, segs, *mats) -> bool:
    """kernels/lora_v3.hip: ranks 16/32/64, up to 64 stacked adapter rows, 8-element aligned
    rows and segments, contiguous f32 adapter weights (checked by the caller)."""
    return (USE_V3 and r in (16, 32, 64) and R % 16 == 0 and R <= 64
            and all(s[0] % 8 == 0 and s[1] % 8 == 0 for s in segs)
            and all(m.stride(1) == 1 and m.stride(0) % 8 == 0 for m in mats))


def _lora3_down(x2d, A, Z, p, seed):
    """Z += drop(x) A^T (f32 [T, R])."""
    T, K = x2d.shape
    R = A.shape[0]
    cnt = slab = None
    if DETERMINISTIC and x2d.is_cuda:
        slab, cnt = _det_ws(x2d.device, math.ceil(T / 64) * math.ceil(K / 1024) * 64 * R,
                            math.ceil(T / 64))
    native().lora3_down(x2d, x2d.stride(0), A, Z, R, T, K, R, 1.0, int(seed) & 0x7FFFFFFFFFFFFFFF,
                        drop_threshold(p), 1.0 / (1.0 - p) if p > 0 else 1.0, K, 0,
                        None, 0, 0, None if (slab is not None and DET_SPLIT) else cnt, slab)


def _lora3_fwd(x2d, y, A, B, Z, segs, r, scale, p, seed, rope):
    """v3 DOWN, then the v2 UP write-back (its write-back issues the RoPE table loads with the
    output loads).  Returns (y, rope fused).  (Running the memory-bound adapter products on a
    side stream under the frozen-weight GEMM measured +1.7 ms/step and was removed.)"""
    _lora3_down(x2d, A, Z, p, seed)
    fuse = rope is not None and len(segs) <= 4 and _rope_covered(segs, rope[3])
    for i in range(0, len(segs), 4):
        ch = segs[i:i + 4]
        mask = sum(1 << j for j, sg in enumerate(ch) if sg[0] + sg[1] <= rope[3]) if fuse else 0
        _lora2(2, 1, B, Z, y, y.stride(0), 1, scale, T=x2d.shape[0], J=r, split=1,
               segs4=[(b_off * r, r_off, n_off, n_len) for (n_off, n_len, r_off, b_off) in ch],
               rope=(rope[1], rope[2], rope[0], mask) if fuse else None)
    return y, fuse


# LUMEN_LORA_FOLD (default on): the forward UP product is folded into the frozen-weight GEMM as
# 64 extra K columns, y = [x | Z | 0] [W | s B_bd | 0]^T, for persistent 16-bit weights whose
# input producer wrote x into the first K columns of a [T, K + 64] buffer (RMSNorm for q|k|v,
# flash attention for o): the 16-bit read-modify-write of y disappears; RoPE then runs as its
# own pass over q|k.
FOLD = _os.environ.get("LUMEN_LORA_FOLD", "1") != "0"
FOLD_KP = 64


def fold_operand(x2d: torch.Tensor, K: int) -> Optional[torch.Tensor]:
    """The [T, K + FOLD_KP] operand behind a producer's [T, K] view of it, else None."""
    if (x2d.dim() == 2 and x2d.shape[1] == K and x2d.stride(1) == 1
            and x2d.stride(0) == K + FOLD_KP and x2d.is_cuda):
        return x2d.as_strided((x2d.shape[0], K + FOLD_KP), (K + FOLD_KP, 1))
    return None


def _dy_tw(segs, T: int) -> int:
    """dY rows per block of lora3_dy: 256 unless that leaves fewer than 512 blocks (dZ / dB
    atomics grow as the tile shrinks: 128 only for narrow outputs such as o_proj)."""
    if DY_TW:
        return DY_TW
    cols = sum(math.ceil(s[1] / 256) for s in segs)
    return 256 if cols * math.ceil(T / 256) >= 512 else 128


def lora_fwd_native(x2d, y, A, B, segs: Sequence[Seg], r, scale, p, seed, train: bool = False,
                    rope=None):
    """Z = drop(x) A^T (f32 [T,R]); y[:, seg] += scale * Z[:, rseg] B_seg^T (in place).

    ``rope`` = (pos int32 [T], cos, sin, ncols): also rotate columns [0, ncols) of y (q|k heads,
    head dim 128) in the same pass when adapter segments cover exactly that range.  Returns
    (Z, rope_done)."""
    T, K = x2d.shape
    R = A.shape[0]
    v3 = (_v3_ok(r, R, segs, x2d, y) and K % 8 == 0
          and A.is_contiguous() and B.is_contiguous() and A.dtype == B.dtype == torch.float32)
    Ntot = y.shape[1]
    act = DTYPE_CODE[x2d.dtype]
    Z = _zeros(T, R, device=x2d.device, train=train)
    if v3:
        y, fuse = _lora3_fwd(x2d, y, A, B, Z, segs, r, scale, p, seed, rope)
        return Z, fuse
    if _v2_ok(r, R, x2d):
        _lora2(0, 1, x2d, A, Z, R, 1, 1.0, T, R, _split(math.ceil(T / 64), K, 256),
               [(0, 0, 0, K)], seed, p, K)
    else:
        _lora_gemm(act, 1, x2d, A, Z, K, K, R, 1, 1.0, [(0, 0, 0, T, R, K)],
                   _ksplit(T, R, K, _bn(R)), seed, p, K)
    if _v2_ok(r, R, x2d, y) and all(s[0] % 8 == 0 and s[1] % 8 == 0 for s in segs):
        fuse = rope is not None and len(segs) <= 4 and _rope_covered(segs, rope[3])
        for i in range(0, len(segs), 4):
            ch = segs[i:i + 4]
            rp = None
            if fuse:
                mask = sum(1 << j for j, sg in enumerate(ch) if sg[0] + sg[1] <= rope[3])
                rp = (rope[1], rope[2], rope[0], mask)
            _lora2(2, 1, B, Z, y, y.stride(0), 1, scale, T, r, 1,
                   [(b_off * r, r_off, n_off, n_len) for (n_off, n_len, r_off, b_off) in ch],
                   rope=rp)
        return Z, fuse
    segs6 = [(r_off, b_off * r, n_off, T, n_len, r) for (n_off, n_len, r_off, b_off) in segs]
    for i in range(0, len(segs6), 4):
        _lora_gemm(act, 6, Z, B, y, R, r, Ntot, 1, scale, segs6[i:i + 4], 1)
    return Z, False


def _rope_covered(segs, ncols: int) -> bool:
    """Adapter segments tile [0, ncols) exactly in 128-column heads (fused RoPE precondition)."""
    cov = sorted((s[0], s[0] + s[1]) for s in segs if s[0] < ncols)
    cur = 0
    for a, b in cov:
        if a != cur or b > ncols or a % 128 or b % 128:
            return False
        cur = b
    return cur == ncols


def lora_bwd_native(dy, x2d, A, B, Z, dx, segs: Sequence[Seg], r, scale, p, seed,
                    need_dA=True, need_dB=True, dx_fn=None):
    """Returns (dA, dB); adds dZ A into dx in place.  ``dx_fn`` (with dx None): produces the
    frozen path's input gradient (a fresh contiguous [T, K] tensor) when the adapter pass is
    ready for it -- with ``LUMEN_LORA_BWD_OVERLAP=1`` the dZ / dB pass runs on a side stream
    beside that GEMM."""
    T, K = x2d.shape
    R = A.shape[0]
    Ntot = dy.shape[1]
    act = DTYPE_CODE[dy.dtype]
    dev = dy.device
    v2 = _v2_ok(r, R, x2d, dy)
    v3 = (v2 and _v3_ok(r, R, segs, x2d, dy) and K % 8 == 0 and A.is_contiguous()
          and B.is_contiguous() and A.dtype == B.dtype == torch.float32)
    v3 = v3 and (dx is None or _v3_ok(r, R, segs, dx))
    # dA / dB accumulate straight into the parameters' .grad (views of the engine's flat f32
    # gradient buffer) when they exist: no zero-filled temporaries and no autograd add kernels
    direct = v2 and DIRECT_GRAD and _direct_ok(A) and _direct_ok(B)
    if v3:
        return _lora3_bwd(dy, x2d, A, B, Z, dx, segs, r, scale, p, seed, need_dA, need_dB, direct,
                          dx_fn)
    if dx_fn is not None:
        dx = dx_fn()
    nA = R * K if need_dA and not direct else 0
    nB = B.shape[0] * r if need_dB and not direct else 0
    ws = _zeros(T * R + nA + nB, device=dev)
    dZ = ws[:T * R].view(T, R)
    if v2:
        for i in range(0, len(segs), 4):
            ch = segs[i:i + 4]
            _lora2(0, 0, dy, B, dZ, R, 1, scale, T, r,
                   _split(math.ceil(T / 64) * len(ch), max(s[1] for s in ch), 256),
                   [(n_off, b_off * r, r_off, n_len) for (n_off, n_len, r_off, b_off) in ch])
    else:
        s2 = [(n_off, b_off * r, r_off, T, r, n_len) for (n_off, n_len, r_off, b_off) in segs]
        for i in range(0, len(s2), 4):
            chunk = s2[i:i + 4]
            _lora_gemm(act, 2, dy, B, dZ, Ntot, r, R, 1, scale, chunk,
                       _ksplit(T, r, max(s[5] for s in chunk), 16, len(chunk)))
    dA = dB = None
    if need_dA:
        dA = A.grad if direct else ws[T * R:T * R + nA].view(R, K)
        if v2:
            _lora2(1, 1, x2d, dZ, dA, 1, K, 1.0, T, R, _split(math.ceil(K / 128), T, 128),
                   [(0, 0, 0, K)], seed, p, K)
        else:
            _lora_gemm(act, 3, dZ, x2d, dA, R, K, K, 1, 1.0, [(0, 0, 0, R, K, T)],
                       _ksplit(R, K, T, 64), seed, p, K)
    if need_dB:
        dB = B.grad if direct else ws[T * R + nA:].view(B.shape[0], r)
        if v2:
            for i in range(0, len(segs), 4):
                ch = segs[i:i + 4]
                _lora2(1, 0, dy, Z, dB, r, 1, scale, T, r,
                       _split(sum(math.ceil(s[1] / 128) for s in ch), T, 128),
                       [(n_off, r_off, b_off * r, n_len) for (n_off, n_len, r_off, b_off) in ch])
        else:
            s4 = [(n_off, r_off, b_off * r, n_len, r, T) for (n_off, n_len, r_off, b_off) in segs]
            for i in range(0, len(s4), 4):
                chunk = s4[i:i + 4]
                _lora_gemm(act, 4, dy, Z, dB, Ntot, R, r, 1, scale, chunk,
                           _ksplit(max(s[3] for s in chunk), r, T, 16, len(chunk)))
    if dx is not None:
        if v2 and _v2_ok(r, R, dx):
            _lora2(2, 0, A, dZ, dx, dx.stride(0), 1, 1.0, T, R, 1, [(0, 0, 0, K)], seed, p, K)
        else:
            _lora_gemm(act, 5, dZ, A, dx, R, K, K, 1, 1.0, [(0, 0, 0, T, K, R)], 1, seed, p, K)
    if direct:
        for prm, need in ((A, need_dA), (B, need_dB)):
            cb = getattr(prm, "_lumen_grad_ready", None)
            if need and cb is not None:
                cb(prm)
        return None, None
    return dA, dB


def _lora3_bwd(dy, x2d, A, B, Z, dx, segs, r, scale, p, seed, need_dA, need_dB, direct,
               dx_fn=None):
    """v3 backward: ONE pass over dY for dZ and dB (lora3_dy), dA from the dropped-out input
    (v2 WGRAD), dx += drop'(dZ A) lane-local (lora3_up mode 5)."""
    T, K = x2d.shape
    R = A.shape[0]
    dev = dy.device
    nat = native()
    nA = R * K if need_dA and not direct else 0
    nB = B.shape[0] * r if not direct or not need_dB else 0  # dB target even when unused
    ws = _zeros(T * R + nA + nB, device=dev)
    dZ = ws[:T * R].view(T, R)
    dB = B.grad if (direct and need_dB) else ws[T * R + nA:].view(B.shape[0], r)

    def dy_pass():
        for i in range(0, len(segs), 4):  # one pass over dY: dZ and dB
            ch = segs[i:i + 4]
            tw_ = _dy_tw(ch, T)
            ws = cnt = None
            if DETERMINISTIC:
                gx = math.ceil(max(sg[1] for sg in ch) / 256)
                gy = math.ceil(T / tw_)
                ns = len(ch)
                ws, cnt = _det_ws(dev, ns * gy * gx * tw_ * r + ns * gx * gy * 256 * r,
                                  ns * (gx + gy))
            nat.lora3_dy(dy, dy.stride(0), B, r, Z, R, dZ, R, dB, T, tw_, scale,
                         [(n_off, r_off, b_off, n_len) for (n_off, n_len, r_off, b_off) in ch],
                         ws, None if DET_SPLIT else cnt)

    if dx_fn is not None and BWD_OVERLAP and dy.is_cuda:
        # the dY pass (memory-bound, f32 atomics) beside the input-gradient GEMM (MFMA-bound):
        # every operand was produced on the main stream before the fork, and the main stream
        # waits for the side stream before anything reads dZ / dB or frees them
        main = torch.cuda.current_stream(dev)
        side = _side_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            dy_pass()
        dx = dx_fn()
        main.wait_stream(side)
    else:
        dy_pass()
        if dx_fn is not None:
            dx = dx_fn()
    dA = None
    if need_dA:
        dA = A.grad if direct else ws[T * R:T * R + nA].view(R, K)
    if need_dA and dx is None and DXA and DETERMINISTIC and x2d.is_cuda:
        # no input gradient wanted (the first layer): the fused pass still computes dA, its
        # deterministic sum, and updates a throwaway dx (the atomic WGRAD fallback below would
        # make dA order-dependent)
        dx = torch.empty_like(x2d)
    if need_dA and dx is not None and DXA:
        # one pass over the [T, K] rows: dA from the staged x tiles, dx updated lane-locally
        tw = DXA_TW or (256 if math.ceil(K / 128) * math.ceil(T / 256) >= 512 else 128)
        slot = _DELTA_SLOT[0]
        delta = None
        if slot is not None and R == 16 and K % 128 == 0 and dx.shape == x2d.shape:
            delta = torch.empty(K // 128, T, device=dev, dtype=torch.float32)
        ws = cnt = None
        if DETERMINISTIC:
            ws, cnt = _det_ws(dev, math.ceil(K / 128) * math.ceil(T / tw) * 128 * R,
                              math.ceil(K / 128))
        nat.lora3_dxa(x2d, dx, dZ, A, dA, tw, int(seed) & 0x7FFFFFFFFFFFFFFF, drop_threshold(p),
                      1.0 / (1.0 - p) if p > 0 else 1.0, K, 0, delta, ws,
                      None if DET_SPLIT else cnt)
        if delta is not None:
            slot["delta"], slot["key"] = delta, (dx.data_ptr(), dx._version)
    else:
        if need_dA:
            _lora2(1, 1, x2d, dZ, dA, 1, K, 1.0, T, R, _split(math.ceil(K / 128), T, 128),
                   [(0, 0, 0, K)], seed, p, K)
        if dx is not None:
            nat.lora3_up(0, dx, dx.stride(0), dZ, R, A, K, T, R, 1.0,
                         int(seed) & 0x7FFFFFFFFFFFFFFF, drop_threshold(p),
                         1.0 / (1.0 - p) if p > 0 else 1.0, K, 0, [(0, 0, 0, K)],
                         None, None, None, 0)
    if direct:
        for prm, need in ((A, need_dA), (B, need_dB)):
            cb = getattr(prm, "_lumen_grad_ready", None)
            if need and cb is not None:
                cb(prm)
        return None, None
    return dA, (dB if need_dB else None)


DIRECT_GRAD = _os.environ.get("LUMEN_LORA_DIRECT_GRAD", "1") != "0"
# the backward's dZ / dB pass on a side stream beside the input-gradient GEMM (opt-in A/B)
BWD_OVERLAP = _os.environ.get("LUMEN_LORA_BWD_OVERLAP", "0") == "1"
_side_streams: dict = {}


def _side_stream(dev) -> "torch.cuda.Stream":
    s = _side_streams.get(dev)
    if s is None:
        s = _side_streams[dev] = torch.cuda.Stream(device=dev)
    return s


def _direct_ok(prm: torch.Tensor) -> bool:
    g = prm.grad
    return (getattr(prm, "_lumen_direct_grad", False) and g is not None
            and g.dtype == torch.float32 and g.is_contiguous() and g.shape == prm.shape)


# ----------------------------------------------------------------------------------------------
# autograd
# ----------------------------------------------------------------------------------------------

class _LoraLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2d, weight_fn, bias, A, B, segs, r, scale, p, seed, w_param, wt_fn, train,
                rope, fold=None):
        ctx.train = train
        W = weight_fn() if fold is None else None

        def gemm():
            y_ = torch.matmul(x2d, W.t())
            if bias is not None:
                y_.add_(bias)
            return y_

        # autograd runs Function.forward with grad disabled: the training flag is passed in
        if fold is not None:
            T, K = x2d.shape
            R = A.shape[0]
            xe = fold_operand(x2d, K)
            Z = _zeros(T, R, device=x2d.device, train=ctx.train)
            _lora3_down(x2d, A, Z, p, seed)
            native().lora3_z_tail(Z, xe, K, FOLD_KP)
            y = torch.matmul(xe, fold.t())
            if bias is not None:
                y.add_(bias)
            rope_done = False
        else:
            y = gemm()
            Z, rope_done = lora_fwd_native(x2d, y, A, B, segs, r, scale, p, seed,
                                           train=ctx.train, rope=rope)
        if rope is not None and not rope_done:
            _rope_(y, rope, inverse=False)
        ctx.rope = rope
        ctx.delta_slot = getattr(x2d, "_lumen_delta_slot", None) if DELTA_HANDOFF else None
        ctx.weight_fn = weight_fn
        ctx.wt_fn = wt_fn
        ctx.meta = (segs, r, scale, p, seed)
        ctx.w_grad = w_param is not None and w_param.requires_grad
        ctx.b_grad = bias is not None and bias.requires_grad
        ctx.save_for_backward(x2d, A, B, Z)
        return y

    @staticmethod
    def backward(ctx, dy):
        x2d, A, B, Z = ctx.saved_tensors
        segs, r, scale, p, seed = ctx.meta
        dy = dy.contiguous()
        if ctx.rope is not None and not getattr(dy, "_lumen_rope_undone", False):
            # y was rotated in the forward: d(pre-rope) = inverse rotation of the incoming grad
            # (already done when the flash-attention backward produced it, _lumen_rope_undone).
            # In place when the grad is a scratch buffer nothing else reads (the flash-attention
            # backward's fresh dQKV, marked), otherwise on a copy.
            if not getattr(dy, "_lumen_scratch", False):
                dy = dy.clone()
            _rope_(dy, ctx.rope, inverse=True)
        got = {}

        def dx_fn():
            got["dx"] = _input_grad(ctx, dy)
            return got["dx"]

        _IN_BACKWARD[0] = True
        _DELTA_SLOT[0] = ctx.delta_slot
        try:
            dA, dB = lora_bwd_native(dy, x2d, A, B, Z, None, segs, r, scale, p, seed,
                                     ctx.needs_input_grad[3], ctx.needs_input_grad[4],
                                     dx_fn=dx_fn if ctx.needs_input_grad[0] else None)
        finally:
            _IN_BACKWARD[0] = False
            _DELTA_SLOT[0] = None
        dx = got.get("dx")
        dw =torch.matmul(dy.t(), x2d) if ctx.w_grad else None
        db = dy.sum(0) if ctx.b_grad else None
        return dx, None, db, dA, dB, None, None, None, None, None, dw, None, None, None, None


class _Linear(torch.autograd.Function):
    """Plain (frozen or trainable) linear whose weight is re-fetched at backward."""

    @staticmethod
    def forward(ctx, x2d, weight_fn, bias, w_param, wt_fn):
        W = weight_fn()
        y = mm_nt(x2d, W)
        if bias is not None:
            y.add_(bias)
        ctx.weight_fn = weight_fn
        ctx.wt_fn = wt_fn
        ctx.w_grad = w_param is not None and w_param.requires_grad
        ctx.b_grad = bias is not None and bias.requires_grad
        ctx.save_for_backward(x2d if ctx.w_grad else torch.empty(0))
        return y

    @staticmethod
    def backward(ctx, dy):
        (x2d,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = _input_grad(ctx, dy) if ctx.needs_input_grad[0] else None
        dw = torch.matmul(dy.t(), x2d) if ctx.w_grad else None
        db = dy.sum(0) if ctx.b_grad else None
        return dx, None, db, dw, None


def _rope_(x2d, rope, inverse: bool):
    """RoPE over columns [0, ncols) of x2d in place (rope = (pos, cos, sin, ncols), D = 128)."""
    from .rope import _neg

    pos, cos, sin, ncols = rope
    native().rope_inplace(x2d, pos, cos, _neg(sin) if inverse else sin, x2d.shape[0],
                          x2d.stride(0), ncols // 128, 128)


def _input_grad(ctx, dy):
    """dX = dY @ W, as the TN GEMM dY @ (W^T)^T when the layer keeps a transposed copy."""
    Wt = ctx.wt_fn() if ctx.wt_fn is not None else None
    if Wt is not None:
        return mm_nt(dy, Wt)
    return torch.matmul(dy, ctx.weight_fn())


def linear(x: torch.Tensor, weight_fn, bias: Optional[torch.Tensor] = None,
           w_param: Optional[torch.Tensor] = None, wt_fn=None) -> torch.Tensor:
    shp = x.shape
    x2d = x if x.dim() == 2 else x.reshape(-1, shp[-1])
    if use_native(x2d):
        y = _Linear.apply(x2d.contiguous(), weight_fn, bias, w_param, wt_fn)
    else:
        y = F.linear(x2d, _frozen(weight_fn()), bias)
    # 2-D in -> return the Function output itself (not a view): a view would make a later
    # in-place op on it (RoPE on the fused QKV buffer) go through autograd's CopySlices
    return y if x.dim() == 2 else y.view(*shp[:-1], y.shape[-1])


def _frozen(W: torch.Tensor) -> torch.Tensor:
    # autograd must not save the Parameter object itself: ZeRO-3 swaps param.data when it
    # releases a gathered unit; a detached alias keeps the gathered storage alive instead
    return W if W.requires_grad else W.detach()


def lora_linear(x: torch.Tensor, weight_fn, bias: Optional[torch.Tensor], A: torch.Tensor,
                B: torch.Tensor, segs: List[Seg], r: int, scale: float, p: float, seed: int,
                w_param: Optional[torch.Tensor] = None, wt_fn=None, rope=None,
                fold: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``rope`` (GPU path only) = (pos int32 [T], cos, sin, ncols): the output's columns
    [0, ncols) come back rotated (RoPE fused into the adapter write-back when possible).
    ``fold`` = the [N, K + 64] extended weight [W | s B_bd | 0] (x must then be the [T, K] view
    of a [T, K + 64] buffer, see ``fold_operand``)."""
    shp = x.shape
    x2d = x if x.dim() == 2 else x.reshape(-1, shp[-1])
    # the adapter kernels take 16-bit activations (the training / serving dtypes); an fp32
    # model on the GPU (--dtype fp32) runs the adapter products in torch
    if use_native(x2d) and x2d.dtype != torch.float32:
        if fold is not None and fold_operand(x2d, x2d.shape[1]) is None:
            fold = None
        y = _LoraLinear.apply(x2d if fold is not None else x2d.contiguous(), weight_fn, bias, A,
                              B, segs, r, scale, p, seed, w_param, wt_fn,
                              torch.is_grad_enabled(), rope, fold)
    else:
        y = lora_linear_ref(x2d, _frozen(weight_fn()), bias, A, B, segs, r, scale, p, seed)
        if rope is not None:   # the caller expects rotated q|k columns back
            y = _rope_ref_cols(y, rope)
    return y if x.dim() == 2 else y.view(*shp[:-1], y.shape[-1])


def _rope_ref_cols(y: torch.Tensor, rope) -> torch.Tensor:
    """Torch RoPE over columns [0, ncols) (128-wide heads) at positions ``pos`` (out of place)."""
    from .rope import _rotate_ref

    pos, cos_t, sin_t, ncols = rope
    T = y.shape[0]
    p = pos.long()
    head = y[:, :ncols].reshape(T, ncols // 128, 128).transpose(0, 1)
    rot = _rotate_ref(head, cos_t[p], sin_t[p]).transpose(0, 1).reshape(T, ncols)
    return torch.cat([rot, y[:, ncols:]], 1)


def lora_linear_ref(x2d, W, bias, A, B, segs, r, scale, p, seed):
    y = F.linear(x2d, W, bias)
    xd = _apply_dropout_ref(x2d, p, seed)
    Z = xd.float() @ A.float().t()
    parts = []
    cur = 0
    for (n_off, n_len, r_off, b_off) in sorted(segs):
        if n_off > cur:
            parts.append(torch.zeros(x2d.shape[0], n_off - cur, device=x2d.device))
        parts.append(scale * (Z[:, r_off:r_off + r] @ B[b_off:b_off + n_len].float().t()))
        cur = n_off + n_len
    if cur < y.shape[1]:
        parts.append(torch.zeros(x2d.shape[0], y.shape[1] - cur, device=x2d.device))
    delta = torch.cat(parts, 1)
    return (y.float() + delta).to(y.dtype)
