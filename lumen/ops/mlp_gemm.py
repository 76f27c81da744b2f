"""Host side of the hand-written training-shape GEMM with fused SwiGLU epilogues
(``kernels/mlp_gemm.hip``): split-tail workspaces and the call.

``mlp_gemm(epi, x, w, c, act=None, gu=None)``:
  * epi 0: c[M, N] = x @ w^T;
  * epi 1: c = gu = x @ w^T (w = [gate | up] rows), act = silu(g) * u;
  * epi 2: c = dgu from dact = x @ w^T (x = dout, w = Wd^T) and the saved gu.
When the last wave of 256 x 256 tiles fills at most half the CUs it runs split in two k halves
(f32 partial slabs, last-arriver sum), so a 5.375-wave GEMM costs ~5.5 tile times, not 6."""
from __future__ import annotations

import os
from typing import Optional

import torch

from ._native import native

GROUP_M = int(os.environ.get("LUMEN_MLP_GEMM_GROUP_M", "4"))
SPLIT_TAIL = os.environ.get("LUMEN_MLP_GEMM_SPLIT", "1") != "0"
_ws: dict = {}
_cus: dict = {}


def _cu_count(dev) -> int:
    n = _cus.get(dev)
    if n is None:
        n = _cus[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return n


def _workspace(dev, split: int):
    """(slab workspace, ticket counters) per (device, stream): slabs and tickets of launches on
    different streams never interleave; counters stay zeroed between launches."""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    got = _ws.get(key)
    if got is None or got[1].numel() < split:
        n = max(split, 128)
        got = (torch.empty(n * 2 * 65536, dtype=torch.float32, device=dev),
               torch.zeros(n, dtype=torch.int32, device=dev))
        _ws[key] = got
    return got


def mlp_gemm(epi: int, x: torch.Tensor, w: torch.Tensor, c: torch.Tensor,
             act: Optional[torch.Tensor] = None, gu: Optional[torch.Tensor] = None,
             group_m: Optional[int] = None, split: Optional[bool] = None) -> torch.Tensor:
    C = native()
    M, K = x.shape
    n = w.shape[0]
    s = 0
    if (SPLIT_TAIL if split is None else split) and x.is_cuda:
        s = int(C.mlp_gemm_split(M, n, K, epi, _cu_count(x.device)))
    if s:
        ws, cnt = _workspace(x.device, s)
        C.mlp_gemm(epi, x, w, c, act, gu, GROUP_M if group_m is None else group_m, ws, cnt, s)
    else:
        C.mlp_gemm(epi, x, w, c, act, gu, GROUP_M if group_m is None else group_m)
    return c
