"""Multi-adapter serving: several PEFT LoRA adapters over one un-merged base model (SURVEY K27,
the reference's declared vLLM ``--enable-lora``).

Each request picks an adapter by name (OpenAI ``model`` field); a batch mixes requests of
different adapters and of the base model.  Instead of punica-style per-segment kernels with
data-dependent shapes, every adapted projection keeps its adapters stacked:

    A_all [S * R, in]   B_all [out, S * R]   (slot s owns rows / columns s*R .. s*R+R, scale folded)

and a step computes  Z = x A_all^T  ->  Z *= mask(token's slot)  ->  y += Z B_all^T  with two
skinny hipBLASLt GEMMs.  Shapes depend only on the slot count, so the decode path stays
capturable in hipGraphs (the per-token slot ids are one more static input).  The extra work is
S * R extra GEMM columns (S = 4 slots x R = 48 for q|k|v = 192 columns next to 12288), a few
percent of the base projection.  Slot 0 is "no adapter" (its rows are zero).

Tensor parallelism follows the base weights: column-parallel q|k|v / gate|up keep A whole and
slice B by output rows; row-parallel o / down slice A by input columns and all-reduce the small
Z before the B product.
"""
from __future__ import annotations

import json
import os
from typing import Callable, Dict, List, Optional

import torch

_HF = {"q": "self_attn.q_proj", "k": "self_attn.k_proj", "v": "self_attn.v_proj",
       "o": "self_attn.o_proj", "gate": "mlp.gate_proj", "up": "mlp.up_proj",
       "down": "mlp.down_proj"}


def read_peft(path: str):
    """(r, scale, {key: tensor}) of a PEFT adapter dir (safetensors, loaded without pickle)."""
    from safetensors.torch import load_file

    with open(os.path.join(path, "adapter_config.json")) as f:
        c = json.load(f)
    r = int(c["r"])
    scale = float(c.get("lora_alpha", 2 * r)) / r
    return r, scale, load_file(os.path.join(path, "adapter_model.safetensors"))


class _Proj:
    """Stacked adapters of one (fused) projection of one layer."""

    def __init__(self, A: torch.Tensor, B: torch.Tensor, row_parallel: bool):
        self.A, self.B, self.row_parallel = A, B, row_parallel


class MultiLoRA:
    def __init__(self, cfg, adapters: Dict[str, str], max_loras: int, tp_rank: int, tp_size: int,
                 device, dtype):
        if len(adapters) > max_loras:
            raise ValueError(f"{len(adapters)} adapters > max_loras={max_loras}")
        self.names: List[str] = list(adapters)
        self.slots = max_loras + 1                    # slot 0 = base model (no adapter)
        nh, nkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        H, F = cfg.hidden_size, cfg.intermediate_size
        lq, lk, lf = nh * D // tp_size, nkv * D // tp_size, F // tp_size
        r_max = 0
        loaded = []
        for name in self.names:
            r, scale, sd = read_peft(adapters[name])
            r_max = max(r_max, r)
            loaded.append((r, scale, sd))
        self.r = r_max
        S, R = self.slots, r_max
        L = cfg.num_hidden_layers
        # output segments per fused projection: (segment name, rows in the full weight, local
        # row range offset) ; input dim (full / local)
        layout = {
            "qkv": ([("q", nh * D), ("k", nkv * D), ("v", nkv * D)], H, False),
            "o": ([("o", H)], nh * D, True),
            "gate_up": ([("gate", F), ("up", F)], H, False),
            "down": ([("down", H)], F, True),
        }
        self.layers: List[Dict[str, _Proj]] = []
        self.present = set()
        for li in range(L):
            per: Dict[str, _Proj] = {}
            for proj, (segs, k_in, row_par) in layout.items():
                nseg = len(segs)
                k_loc = k_in // tp_size if row_par else k_in
                n_out = sum(n for _, n in segs) // (1 if row_par else tp_size)
                A = torch.zeros(S * nseg * R, k_loc, dtype=dtype)
                B = torch.zeros(n_out, S * nseg * R, dtype=dtype)
                any_set = False
                for slot, (r, scale, sd) in enumerate(loaded, start=1):
                    row0 = 0
                    for si, (seg, n_full) in enumerate(segs):
                        key = f"base_model.model.model.layers.{li}.{_HF[seg]}.lora_"
                        n_loc = n_full if row_par else n_full // tp_size
                        if key + "A.weight" in sd:
                            a = sd[key + "A.weight"].float()            # [r, in]
                            b = sd[key + "B.weight"].float() * scale    # [out, r]
                            if row_par:
                                a = a[:, tp_rank * k_loc:(tp_rank + 1) * k_loc]
                            else:
                                b = b[tp_rank * n_loc:(tp_rank + 1) * n_loc]
                            c0 = (slot * nseg + si) * R
                            A[c0:c0 + r] = a.to(dtype)
                            B[row0:row0 + n_loc, c0:c0 + r] = b.to(dtype)
                            any_set = True
                        row0 += n_loc
                if any_set:
                    self.present.add(proj)
                    per[proj] = _Proj(A.to(device).contiguous(), B.to(device).contiguous(), row_par)
            self.layers.append(per)
        # column -> slot map of the stacked Z, per projection width
        self._col_slot: Dict[int, torch.Tensor] = {}
        self.device = device
        self.dtype = dtype

    def slot_of(self, name: Optional[str]) -> int:
        if not name or name not in self.names:
            return 0
        return self.names.index(name) + 1

    def mask(self, ids: torch.Tensor, nseg: int) -> torch.Tensor:
        """[T, S*nseg*R] 0/1 mask keeping each token's own slot columns."""
        w = self.slots * nseg * self.r
        cs = self._col_slot.get(nseg)
        if cs is None:
            cs = (torch.arange(w, device=self.device) // (nseg * self.r)).to(torch.int32)
            self._col_slot[nseg] = cs
        return (cs[None, :] == ids.to(torch.int32)[:, None]).to(self.dtype)

    def apply(self, layer: int, proj: str, x: torch.Tensor, y: torch.Tensor, masks: dict,
              allreduce: Optional[Callable[[torch.Tensor], torch.Tensor]] = None) -> None:
        """y += (x A^T * mask) B^T for one projection (in place); no-op when absent.
        ``allreduce`` sums the row-parallel partial Z over the TP group (the runner's: custom
        all-reduce inside graphs, RCCL otherwise)."""
        p = self.layers[layer].get(proj)
        if p is None:
            return
        z = torch.matmul(x, p.A.t())
        if p.row_parallel and allreduce is not None:
            allreduce(z)
        nseg = p.A.shape[0] // (self.slots * self.r)
        z.mul_(masks[nseg])
        y.add_(torch.matmul(z, p.B.t()))
