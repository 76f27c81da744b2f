"""Attention ops for training and serving.

* Training (head_dim 128): the HIP flash-attention kernels (``kernels/flash_attn.hip``) read q/k/v
  straight from the fused token-major QKV buffer (``flash_attention_qkv``); other head dims use
  torch SDPA over head-major q/k/v (``causal_attention``).
* Serving decode: the paged-KV HIP kernel (``kernels/paged_attention.hip``, ``paged_decode``).
* Serving prefill -- whole prompts, chunks of long prompts and the prefill part of mixed
  prefill+decode steps: ``flash_attention_paged``, the 32x32x16 flash forward reading keys /
  values from the paged cache through block tables, queries offset by the cached context.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from ._native import native, use_native


def causal_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                     scale: Optional[float] = None) -> torch.Tensor:
    """q [B,nh,S,D], k/v [B,nkv,S,D] -> [B*S, nh*D] (token-major)."""
    B, nh, S, D = q.shape
    nkv = k.shape[1]
    if nkv != nh:
        if q.is_cuda:
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale,
                                               enable_gqa=True)
        else:
            rep = nh // nkv
            o = F.scaled_dot_product_attention(q, k.repeat_interleave(rep, 1),
                                               v.repeat_interleave(rep, 1), is_causal=True,
                                               scale=scale)
    else:
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale)
    return o.transpose(1, 2).reshape(B * S, nh * D)


_merge_counters: dict = {}
# Fused split-context merge (two-pass kernel only): measured neutral in decode steps (batch 1:
# 3.857 vs 3.865 ms ITL, profiles/r02_serve); callers may still ask for it (``fused_merge``).
# decode kernel: 0 = two-pass; 1 = single-pass (K and V streamed together, online softmax per
# row group); 2 = single-pass with workgroup-uniform block ids and non-temporal K / V loads
# (used where the block size equals the kernel's rows per step, else 1); 3 = 2 software-pipelined
# (two register sets, the next iteration's K / V loads in flight while one is consumed; default,
# profiles/r5_decode)
PA_ONE_PASS = int(os.environ.get("LUMEN_PA_1PASS", "3"))


def _pa_counters(device: torch.device, n: int) -> torch.Tensor:
    """Zeroed int32 arrival counters for the fused split-context merge.  The kernel leaves them
    zeroed, so one buffer per device serves every layer and step; it is allocated before any
    HIP-graph capture (the runner's eager warm-up steps reach here first) and only grows."""
    key = (device.type, device.index)
    c = _merge_counters.get(key)
    if c is None or c.numel() < n:
        c = torch.zeros(max(n, 1 << 16), device=device, dtype=torch.int32)
        _merge_counters[key] = c
    return c


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                 block_tables: torch.Tensor, context_lens: torch.Tensor, max_context: int,
                 scale: float, partition_size: int = 512,
                 fused_merge: Optional[bool] = None, one_pass: Optional[bool] = None) -> torch.Tensor:
    """Single-token attention over a paged KV cache.

    q [num_seqs, nh, D]; caches [num_blocks, nkv, block_size, D]; block_tables [num_seqs,
    max_blocks] int32; context_lens [num_seqs] int32 (number of cached tokens incl. current).
    Contexts longer than ``partition_size`` are split over workgroups; with ``fused_merge`` the
    last partition to finish merges the partials (one launch), else a second kernel does.
    """
    num_seqs, nh, D = q.shape
    nb, nkv, bs, _ = k_cache.shape
    if use_native(q):
        max_parts = max(1, math.ceil(max_context / partition_size))
        out = torch.empty(num_seqs, nh, D, device=q.device, dtype=q.dtype)
        if max_parts > 1:
            tm = torch.empty(num_seqs, nh, max_parts, device=q.device, dtype=torch.float32)
            tl = torch.empty_like(tm)
            to = torch.empty(num_seqs, nh, max_parts, D, device=q.device, dtype=torch.float32)
        else:
            tm = torch.empty(1, 1, 1, device=q.device, dtype=torch.float32)
            tl, to = tm, tm
        one = PA_ONE_PASS if one_pass is None else int(one_pass)
        fused = bool(fused_merge) and not one
        cnt = (_pa_counters(q.device, num_seqs * nkv) if fused and max_parts > 1
               else None)
        # q read in place when its heads are contiguous (a view into the fused qkv rows):
        # no per-layer copy of the decode rows' q
        qk = q if (q.stride(2) == 1 and q.stride(1) == D and q.stride(0) % D == 0
                   and q.data_ptr() % 16 == 0) else q.contiguous()
        native().paged_attention_decode(out, qk, k_cache, v_cache, block_tables,
                                        context_lens, nkv, bs, block_tables.shape[1], scale, tm,
                                        tl, to, partition_size, cnt, one)
        return out
    return paged_decode_ref(q, k_cache, v_cache, block_tables, context_lens, scale)


def paged_decode_ref(q, k_cache, v_cache, block_tables, context_lens, scale):
    num_seqs, nh, D = q.shape
    nkv, bs = k_cache.shape[1], k_cache.shape[2]
    g = nh // nkv
    out = torch.empty_like(q)
    for i in range(num_seqs):
        L = int(context_lens[i])
        nblk = (L + bs - 1) // bs
        blks = block_tables[i, :nblk].long()
        kk = k_cache[blks].permute(1, 0, 2, 3).reshape(nkv, nblk * bs, D)[:, :L].float()
        vv = v_cache[blks].permute(1, 0, 2, 3).reshape(nkv, nblk * bs, D)[:, :L].float()
        qq = q[i].float().view(nkv, g, D)
        s = torch.einsum("hgd,hld->hgl", qq, kk) * scale
        p = torch.softmax(s, -1)
        out[i] = torch.einsum("hgl,hld->hgd", p, vv).reshape(nh, D).to(q.dtype)
    return out


def flash_attention_paged(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                          cu_q, kv_lens, block_tables: torch.Tensor, nh: int, nkv: int,
                          D: int, scale: Optional[float] = None,
                          out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Causal attention of prefill chunks over the paged KV cache.

    q: token-major rows [T, >= nh*D] (e.g. the q part of the fused qkv buffer, already rotated);
    sequence s owns rows cu_q[s]..cu_q[s+1] and sees kv_lens[s] keys (its cached context plus
    this chunk, whose K/V are already in the cache); query row j of s sits at key position
    kv_lens[s] - (cu_q[s+1]-cu_q[s]) + j.  cu_q / kv_lens: int sequences (host) or int32 device
    tensors; block_tables [nseq, max_blocks] int32.  Returns / fills out [T, nh*D]."""
    T = q.shape[0]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if out is None:
        out = torch.empty(T, nh * D, device=q.device, dtype=q.dtype)
    if use_native(q) and D == 128 and k_cache.shape[-1] == 128:
        cu = tuple(int(c) for c in cu_q)
        dev = q.device
        cut = _cu_tensor(cu, dev)
        kl = (kv_lens if isinstance(kv_lens, torch.Tensor)
              else torch.tensor(list(kv_lens), dtype=torch.int32, device=dev))
        kl = kl.to(torch.int32)
        bt = block_tables.to(torch.int32)
        if k_cache.dtype == FP8_KV:
            k_cache, v_cache, bt = _dequant_blocks(k_cache, v_cache, bt, kl, q.dtype)
        native().flash_attn_paged(True, q, k_cache, v_cache, out, cut, kl,
                                  _tiles(cu, 128, dev), bt, nh, nkv, scale)
        return out
    out.copy_(flash_attention_paged_ref(q, k_cache, v_cache, cu_q, kv_lens, block_tables, nh,
                                        nkv, D, scale))
    return out


FP8_KV = torch.float8_e4m3fn  # fp8 KV-cache element type (OCP e4m3fn: gfx950's fp8 converts)
_SCRATCH: dict = {}


def _dequant_blocks(k_cache, v_cache, bt, kv_lens, dtype):
    """fp8 cache -> 16-bit scratch holding only the prefill sequences' blocks (block b of
    sequence s at s * maxb + b), plus the identity block table into it: the prefill kernel's
    LDS-DMA staging moves raw 16-bit rows.  The scratch is reused by every layer and grows."""
    P, maxb = bt.shape
    nb, nkv, bs, D = k_cache.shape
    need = P * maxb
    key = (k_cache.device, dtype, nkv, bs, D)
    scr = _SCRATCH.get(key)
    if scr is None or scr[0].shape[0] < need:
        n = max(need, 256)
        scr = (torch.empty(n, nkv, bs, D, device=k_cache.device, dtype=dtype),
               torch.empty(n, nkv, bs, D, device=k_cache.device, dtype=dtype),
               torch.arange(n, device=k_cache.device, dtype=torch.int32))
        _SCRATCH[key] = scr
    ks, vs, ident = scr
    native().kv_dequant(k_cache, v_cache, ks, vs, bt, kv_lens, maxb)
    return ks, vs, ident[:need].view(P, maxb)


def flash_attention_paged_ref(q, k_cache, v_cache, cu_q, kv_lens, block_tables, nh, nkv, D,
                              scale=None):
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    cu = [int(c) for c in cu_q]
    kl = [int(x) for x in kv_lens]
    bs = k_cache.shape[2]
    g = nh // nkv
    outs = []
    for s in range(len(kl)):
        a, b = cu[s], cu[s + 1]
        n, L = b - a, kl[s]
        nblk = (L + bs - 1) // bs
        blks = block_tables[s, :nblk].long()
        kk = k_cache[blks].permute(1, 0, 2, 3).reshape(nkv, nblk * bs, D)[:, :L].float()
        vv = v_cache[blks].permute(1, 0, 2, 3).reshape(nkv, nblk * bs, D)[:, :L].float()
        qq = q[a:b, :nh * D].float().view(n, nkv, g, D)
        sc = torch.einsum("nhgd,hld->hgnl", qq, kk) * scale
        qpos = torch.arange(L - n, L, device=q.device)[:, None]
        kpos = torch.arange(L, device=q.device)[None, :]
        sc = sc.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(sc, -1)
        o = torch.einsum("hgnl,hld->nhgd", p, vv).reshape(n, nh * D)
        outs.append(o.to(q.dtype))
    return torch.cat(outs, 0) if outs else q.new_zeros(0, nh * D)


def write_kv_cache(k: torch.Tensor, v: torch.Tensor, k_cache: torch.Tensor,
                   v_cache: torch.Tensor, slot_mapping: torch.Tensor) -> None:
    """k, v: [T, nkv, D] views (row stride may exceed nkv*D); slot_mapping [T] int64."""
    T = slot_mapping.numel()
    if T == 0:
        return
    nb, nkv, bs, D = k_cache.shape
    if use_native(k_cache):
        native().reshape_and_cache(k, v, k_cache, v_cache, slot_mapping, nkv, D, bs,
                                   k.stride(0), v.stride(0))
        return
    sm = slot_mapping.long()
    valid = sm >= 0
    sm = sm[valid]
    blk, off = sm // bs, sm % bs
    k_cache[blk, :, off] = k[valid].to(k_cache.dtype)
    v_cache[blk, :, off] = v[valid].to(v_cache.dtype)


def rope_write_kv(qkv: torch.Tensor, positions: torch.Tensor, nh: int, nkv: int, D: int,
                  cos_t: torch.Tensor, sin_t: torch.Tensor, k_cache: torch.Tensor,
                  v_cache: torch.Tensor, slot_mapping: torch.Tensor) -> None:
    """RoPE on the q and k heads of the fused token-major qkv [T, (nh + 2 nkv) D] in place, then
    the rotated k and v into the paged cache at ``slot_mapping`` (-1 = skip): one HIP kernel
    (``rope_cache_kernel``) on GPU, rope_inplace + write_kv_cache elsewhere."""
    T = qkv.shape[0]
    if T == 0:
        return
    nb, nkv_c, bs, Dc = k_cache.shape
    if use_native(qkv) and D % 16 == 0 and nkv_c == nkv and Dc == D:
        native().rope_cache_write(qkv, positions.to(torch.int32), cos_t, sin_t, k_cache, v_cache,
                                  slot_mapping.to(torch.int64), nh, nkv, D, bs)
        return
    from .rope import rope_inplace

    rope_inplace(qkv, positions, nh + nkv, D, cos_t, sin_t)
    qs, ks = nh * D, nkv * D
    write_kv_cache(qkv[:, qs:qs + ks].view(T, nkv, D), qkv[:, qs + ks:qs + 2 * ks].view(T, nkv, D),
                   k_cache, v_cache, slot_mapping)


# ------------------------------------------------------------------------------------------------
# HIP flash attention over the fused token-major QKV buffer (kernels/flash_attn.hip)
# ------------------------------------------------------------------------------------------------

_TILE_CACHE = {}


def _upload_i32(vals, device) -> torch.Tensor:
    """Small int32 host list -> device without a stream synchronise: a blocking
    ``torch.tensor(..., device=gpu)`` copy waits for every kernel queued before it, which would
    serialise the serving engine's host work (a new chunk layout every step) with the GPU.  The
    pinned staging block is recycled by torch's caching host allocator once the copy is done."""
    h = torch.tensor(vals, dtype=torch.int32)
    if torch.device(device).type != "cuda":
        return h
    return h.pin_memory().to(device, non_blocking=True)


def _tiles(cu: tuple, rows: int, device, heavy_first: bool = True,
           heavy_low: bool = False) -> torch.Tensor:
    """(seq, row start) pairs; heavy_first: causal query tiles (last rows = most keys) first;
    heavy_low: key tiles of the dK/dV kernels (first rows = most queries) first."""
    key = (cu, rows, str(device), heavy_first, heavy_low)
    t = _TILE_CACHE.get(key)
    if t is None:
        lst = []
        for s in range(len(cu) - 1):
            L = cu[s + 1] - cu[s]
            lst += [(s, r) for r in range(0, L, rows)]
        if heavy_low:
            lst.sort(key=lambda x: (x[1], -(cu[x[0] + 1] - cu[x[0]])))
        elif heavy_first:  # causal: the last tiles of a sequence carry the most keys
            lst.sort(key=lambda x: -x[1])
        t = _upload_i32(lst if lst else [(0, 0)], device).reshape(-1)
        if not lst:
            t = t[:0]
        if len(_TILE_CACHE) > 256:
            _TILE_CACHE.clear()
        _TILE_CACHE[key] = t
    return t


def _cu_tensor(cu: tuple, device) -> torch.Tensor:
    key = ("cu", cu, str(device))
    t = _TILE_CACHE.get(key)
    if t is None:
        t = _upload_i32(list(cu), device)
        _TILE_CACHE[key] = t
    return t


def prepare_varlen(cu: tuple, device) -> None:
    """Seed the tile / offset caches for a packed batch's ``cu`` with ONE pinned, non-blocking
    host-to-device copy, before the layer loop: every layer's forward and backward then hits
    the cache instead of building (and synchronously uploading) its tile lists."""
    rows_set = (FA_FWD_ROWS, 64, 128)
    keys = ([("cu", cu, str(device))] + [(cu, r, str(device), True, False) for r in rows_set]
            + [(cu, 64, str(device), True, True)])
    if all(k in _TILE_CACHE for k in keys):
        return
    parts = [list(cu)]
    for rows, low in [(r, False) for r in rows_set] + [(64, True)]:
        lst = []
        for s in range(len(cu) - 1):
            lst += [(s, r) for r in range(0, cu[s + 1] - cu[s], rows)]
        if low:  # dK/dV key tiles, heaviest (lowest) first
            lst.sort(key=lambda x: (x[1], -(cu[x[0] + 1] - cu[x[0]])))
        else:
            lst.sort(key=lambda x: -x[1])
        parts.append([v for t in lst for v in t])
    flat = torch.tensor([v for p in parts for v in p], dtype=torch.int32)
    if torch.cuda.is_available():
        flat = flat.pin_memory()
    dev = flat.to(device, non_blocking=True)
    if len(_TILE_CACHE) > 256:
        _TILE_CACHE.clear()
    o = 0
    for k, p in zip(keys, parts):
        _TILE_CACHE[k] = dev[o:o + len(p)]
        o += len(p)
    _TILE_CACHE[("pin", cu, str(device))] = flat  # host buffer outlives the async copy


import os as _os
# forward: the 32x32x16 MFMA kernel, 32 queries per wave, 128-row tiles (56 vs 71 us for the
# 16x16x32 forms at B8 S512, profiles/r02_fa; those variants were removed)
FA_FWD_MT, FA_FWD_ROWS = 20, 128
# (a 256-query-tile forward, mt 21, measured slower and was removed: profiles/r5_fa)
# backward: 16x16x32 dK/dV (64-key tiles) + 32x32x16 dQ (128-query tiles), or -- while the buffer
# fits -- the dS hand-off pair below
# dS hand-off: the dK/dV kernel stores dS per 64x64 tile and the dQ kernel forms
# dQ = dS K from it, instead of recomputing S = Q K^T and dP = dO V^T (2 of its 3 products).
# Used while the [nh, tiles, 64, 64] 16-bit buffer stays under LUMEN_FA_DS_MB (0 = off).
FA_DS_MB = float(_os.environ.get("LUMEN_FA_DS_MB", "2048"))
# (Measured and removed: an 8-wave 128-key dK/dV kernel, 117.6 vs 108.0 us at B=8 S=512; XCD-
# grouped 1-D tile orders, neutral; the 32x32 dQ kernel forming delta itself, neutral.)


def _ds_offsets(cu: tuple, causal: bool, device):
    """Per-sequence first tile of the dS hand-off buffer and the total tile count."""
    key = ("ds", cu, causal, str(device))
    hit = _TILE_CACHE.get(key)
    if hit is None:
        offs, tot = [], 0
        for s in range(len(cu) - 1):
            n = (cu[s + 1] - cu[s] + 63) // 64
            offs.append(tot)
            tot += n * (n + 1) // 2 if causal else n * n
        hit = (torch.tensor(offs if offs else [0], dtype=torch.int32, device=device), tot)
        _TILE_CACHE[key] = hit
    return hit


DELTA_HANDOFFS = [0]  # backward calls that used a delta handed over by the o_proj backward


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cu, nh, nkv, D, causal, rope=None, scale=None, out_ext=0):
        C = native()
        T = qkv.shape[0]
        q = qkv[:, :nh * D]
        k = qkv[:, nh * D:(nh + nkv) * D]
        v = qkv[:, (nh + nkv) * D:]
        # out_ext > 0: O is the first nh*D columns of a [T, nh*D + out_ext] buffer (the operand
        # of the o_proj's K-extended LoRA GEMM); the kernels take the row stride
        o = torch.empty(T, nh * D + out_ext, device=qkv.device, dtype=qkv.dtype)[:, :nh * D]
        lse = torch.empty(nh, T, device=qkv.device, dtype=torch.float32)
        cut = _cu_tensor(cu, qkv.device)
        scale = 1.0 / math.sqrt(D) if scale is None else scale
        tl = _tiles(cu, FA_FWD_ROWS, qkv.device)
        C.flash_attn(0, causal, FA_FWD_MT, q, k, v, o, lse, cut, tl, nh, nkv, scale, None, None,
                     None, None, None, None, None, None)
        ctx.save_for_backward(qkv, o, lse)
        ctx.meta = (cu, nh, nkv, D, causal, scale)
        ctx.rope = rope
        # delta hand-off: the o_proj backward (lumen.ops.lora, fused dA + dx kernel) may leave
        # delta = rowsum(dO * O) here for exactly the dO this backward receives
        ctx.delta_slot = {}
        o._lumen_delta_slot = ctx.delta_slot
        return o

    @staticmethod
    def backward(ctx, do):
        C = native()
        qkv, o, lse = ctx.saved_tensors
        cu, nh, nkv, D, causal, scale = ctx.meta
        do = do.contiguous()
        T = qkv.shape[0]
        q = qkv[:, :nh * D]
        k = qkv[:, nh * D:(nh + nkv) * D]
        v = qkv[:, (nh + nkv) * D:]
        dqkv = torch.empty_like(qkv)
        dqkv._lumen_scratch = True  # fresh buffer: consumers may transform it in place
        dq = dqkv[:, :nh * D]
        dk = dqkv[:, nh * D:(nh + nkv) * D]
        dv = dqkv[:, (nh + nkv) * D:]
        slot = ctx.delta_slot
        handed = (slot.get("key") == (do.data_ptr(), do._version)
                  and tuple(slot["delta"].shape) == (nh, T))
        delta = (slot.pop("delta") if handed
                 else torch.empty(nh, T, device=qkv.device, dtype=torch.float32))
        DELTA_HANDOFFS[0] += int(handed)
        slot.clear()
        cut = _cu_tensor(cu, qkv.device)
        # dK/dV (which 2, 64-key tiles) and dQ (which 5, 128-query tiles); both undo the
        # forward's RoPE in their dQ / dK epilogues (d(pre-rotation) written directly): the
        # producer of q|k then skips its own inverse-rotation pass
        wkv, rkv, wq, rq = 2, 64, 5, 128
        rp = ctx.rope
        pos, cos, sin = rp if rp is not None else (None, None, None)
        qtiles = _tiles(cu, rq, qkv.device)
        ds_off, ds_total = (_ds_offsets(cu, causal, qkv.device) if FA_DS_MB > 0
                            else (None, 0))
        if ds_off is not None and nh * ds_total * 8192 <= FA_DS_MB * 2 ** 20:
            ds = torch.empty(nh, ds_total, 4096, device=qkv.device, dtype=qkv.dtype)
            if not handed:
                C.flash_attn(1, causal, 1, q, k, v, o, lse, cut, _tiles(cu, 64, qkv.device), nh,
                             nkv, scale, do, None, None, None, delta, None, None, None)
            # dK/dV: low key tiles carry the most (causal) query steps -> launched first
            t7 = _tiles(cu, 64, qkv.device, heavy_low=causal)
            t8 = _tiles(cu, 64, qkv.device)
            C.flash_attn_ds(7, causal, q, k, v, lse, cut, t7, nh, nkv,
                            scale, do, dq, dk, dv, delta, ds, ds_off, ds_total, pos, cos, sin)
            C.flash_attn_ds(8, causal, q, k, v, lse, cut, t8, nh, nkv,
                            scale, do, dq, dk, dv, delta, ds, ds_off, ds_total, pos, cos, sin)
        else:
            if not handed:
                C.flash_attn(1, causal, 1, q, k, v, o, lse, cut, _tiles(cu, 64, qkv.device), nh,
                             nkv, scale, do, None, None, None, delta, None, None, None)
            C.flash_attn(wkv, causal, 1, q, k, v, o, lse, cut, _tiles(cu, rkv, qkv.device), nh,
                         nkv, scale, do, dq, dk, dv, delta, pos, cos, sin)
            C.flash_attn(wq, causal, 1, q, k, v, o, lse, cut, qtiles, nh, nkv,
                         scale, do, dq, dk, dv, delta, pos, cos, sin)
        if rp is not None:
            dqkv._lumen_rope_undone = True
        return dqkv, None, None, None, None, None, None, None, None


KERNEL_D = 128  # head dim of the HIP flash-attention kernels


def _flash_padded(qkv, cu, nh, nkv, D, causal):
    """Head dims below the kernels' 128 (OPT-125m: 64): every head is zero-padded to 128
    columns -- q.k over the padded heads is the same score, P.V leaves the pad columns of O
    zero -- and the kernel runs with the true 1/sqrt(D) scale.  The pad / slice copies are
    differentiated by autograd (their backward is the slice / pad of the gradient)."""
    T = qkv.shape[0]
    H3 = nh + 2 * nkv
    qkvp = F.pad(qkv.view(T, H3, D), (0, KERNEL_D - D)).view(T, H3 * KERNEL_D)
    o = _FlashAttn.apply(qkvp, cu, nh, nkv, KERNEL_D, causal, None, 1.0 / math.sqrt(D))
    return o.view(T, nh, KERNEL_D)[:, :, :D].reshape(T, nh * D)


def flash_attention_qkv(qkv: torch.Tensor, cu_seqlens, nh: int, nkv: int, D: int,
                        causal: bool = True, rope=None, out_ext: int = 0) -> torch.Tensor:
    """Causal attention straight from the fused token-major QKV buffer [T, (nh+2nkv)*D]
    (q/k already rotated); returns O token-major [T, nh*D].  ``cu_seqlens``: sequence offsets.

    ``rope`` = (pos int32 [T], cos, sin) of the rotation the q/k producer applied: the backward
    then returns the gradient w.r.t. the PRE-rotation q/k (marked ``_lumen_rope_undone`` on the
    dQKV tensor so the producer's backward skips its inverse pass)."""
    cu = tuple(int(c) for c in cu_seqlens)
    if use_native(qkv) and D == KERNEL_D:
        return _FlashAttn.apply(qkv, cu, nh, nkv, D, causal, rope, None, out_ext)
    if use_native(qkv) and D < KERNEL_D and D % 8 == 0 and rope is None:
        return _flash_padded(qkv.contiguous(), cu, nh, nkv, D, causal)
    return flash_attention_ref(qkv, cu, nh, nkv, D, causal)


def flash_attention_fresh(qkv: torch.Tensor, cu, nh: int, nkv: int, D: int, scale: float,
                          out: torch.Tensor) -> torch.Tensor:
    """Inference causal attention of whole fresh prompts straight from the rotated fused qkv rows
    [T, (nh + 2 nkv) D] (the training forward kernel, no autograd), into ``out`` [T, nh D]
    (row-strided views allowed)."""
    cu = tuple(int(c) for c in cu)
    T = qkv.shape[0]
    q = qkv[:, :nh * D]
    k = qkv[:, nh * D:(nh + nkv) * D]
    v = qkv[:, (nh + nkv) * D:(nh + 2 * nkv) * D]
    lse = torch.empty(nh, T, device=qkv.device, dtype=torch.float32)
    native().flash_attn(0, True, FA_FWD_MT, q, k, v, out, lse, _cu_tensor(cu, qkv.device),
                        _tiles(cu, FA_FWD_ROWS, qkv.device), nh, nkv, scale, None, None, None,
                        None, None, None, None, None)
    return out


def flash_attention_ref(qkv, cu, nh, nkv, D, causal=True):
    outs = []
    for s in range(len(cu) - 1):
        a, b = cu[s], cu[s + 1]
        n = b - a
        q = qkv[a:b, :nh * D].view(n, nh, D).transpose(0, 1)[None]
        k = qkv[a:b, nh * D:(nh + nkv) * D].view(n, nkv, D).transpose(0, 1)[None]
        v = qkv[a:b, (nh + nkv) * D:].view(n, nkv, D).transpose(0, 1)[None]
        if nkv != nh:
            rep = nh // nkv
            k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
        outs.append(o[0].transpose(0, 1).reshape(n, nh * D))
    return torch.cat(outs, 0)
