"""HBM plan of a ZeRO-3 + LoRA training job, computed without allocating anything.

The runtime decisions that shape a rank's memory are made in three places, each from the HBM it
sees at that moment:

* ``ParamCoordinator._hbm_live_budget`` -- ``stage3_max_live_parameters: "auto"``: gathered
  elements that fit in the free HBM after the shards minus the activation reserve, which picks
  the schedule (``keep`` / ``hybrid`` / ``release``, ``ParamCoordinator.auto_schedule``);
* ``ParamCoordinator.enable_transposes`` (gathered weights) and ``configure_backward_layout``
  (persistent weights): W^T copies for the TN input-gradient GEMMs, only while they leave the
  reserve free;
* ``Trainer._auto_checkpointing``: the cheapest activation-recompute policy whose activations fit
  twice in what is left.

Those call sites use the helpers below, and ``plan_zero3`` replays the same decisions for a
model config, world size and device capacity (e.g. Llama-2-70B at world 8 on 288 GB: BASELINE
config 5) so a plan can be checked on the CPU.  Reference: configs/ds_config_zero3.json:16-37
(stage3_max_live_parameters, offload), SURVEY.md section 7.4.9.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

GiB = 2 ** 30

# 16-bit H-wide rows per token per layer a micro-step keeps for the backward (measured: 14 GB for
# 8 x 512 Llama-2-7B tokens, profiles/r3_*); selective recompute keeps ~0.65 of it
ACT_ROWS_PER_LAYER = 16
SELECTIVE_FRACTION = 0.65
# HIP context, RCCL channels / proxy buffers, allocator slack, GEMM workspaces
RUNTIME_OVERHEAD = 4 * GiB
# LM-head cross-entropy chunk, adapter scratch arena, collective staging
TRANSIENT = 2 * GiB


def activation_reserve(total_bytes: float, env: str = "LUMEN_ZERO3_RESERVE_GB") -> float:
    """HBM the weight-side decisions leave for activations: max(48 GiB, 25% of the device)
    (``env`` overrides, in GiB)."""
    gb = float(os.environ.get(env, "0") or 0)
    return gb * GiB if gb else max(48 * GiB, 0.25 * total_bytes)


def live_budget_elems(free_bytes: float, total_bytes: float, elem_bytes: int) -> int:
    """``stage3_max_live_parameters: "auto"``: gathered elements that fit after the reserve."""
    return max(0, int((free_bytes - activation_reserve(total_bytes)) // max(elem_bytes, 1)))


def transposes_fit(need_bytes: float, gathered_bytes: float, free_bytes: float,
                   total_bytes: float) -> bool:
    """W^T of the resident gathered projections (all or none) next to the gathered copy."""
    return need_bytes + gathered_bytes <= free_bytes - activation_reserve(total_bytes)


def _act_fraction(policy: str, k: int, L: int) -> float:
    """Activations kept under ``policy`` on the first k of L layers, as a fraction of none."""
    if policy == "selective":
        return 1.0 - k * (1.0 - SELECTIVE_FRACTION) / L
    # full on k layers: their inputs only, plus one layer's activations during its recompute
    return (L - k) / L + k / (ACT_ROWS_PER_LAYER * L) + (1.0 / L if k else 0.0)


def _split_policy(policy):
    if isinstance(policy, str) and ":" in policy:
        p, n = policy.split(":", 1)
        return p, int(n)
    return policy, None


def activation_bytes(cfg, tokens: int, policy: str = "none") -> float:
    """Activations a micro-step of ``tokens`` keeps for its backward under a recompute policy
    (``full``: the layer inputs plus one layer's activations during its recompute;
    ``"selective:N"`` / ``"full:N"``: that policy on the first N layers only)."""
    L, H = cfg.num_hidden_layers, cfg.hidden_size
    full = tokens * L * ACT_ROWS_PER_LAYER * H * 2
    if policy in ("none", False, None):
        return float(full)
    if policy is True:
        policy = "selective"
    p, n = _split_policy(policy)
    return float(full * _act_fraction(p, L if n is None else min(n, L), L))


def pick_checkpointing(est_bytes: float, free_bytes: float, selective_ok: bool,
                       n_layers: Optional[int] = None):
    """``--gradient_checkpointing auto``: none when the activations fit twice, else selective
    (where every layer can run it), else full per-layer recompute.  With ``n_layers`` (the
    model takes ``"policy:N"``) only as many layers recompute as the budget needs: the
    recompute cost grows with N, so the fewest that fit."""
    if 2 * est_bytes <= free_bytes:
        return False
    L = n_layers
    for pol in (("selective", "full") if selective_ok else ("full",)):
        if L:
            for k in range(1, L + 1):
                if 2 * est_bytes * _act_fraction(pol, k, L) <= free_bytes:
                    return pol if k == L else f"{pol}:{k}"
        elif pol == "selective" and 2 * SELECTIVE_FRACTION * est_bytes <= free_bytes:
            return "selective"
    return "full"


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def llama_units(cfg, lora_targets=("q_proj", "k_proj", "v_proj", "o_proj"), lora_r: int = 16,
                fold_kp: int = 64) -> List[Dict]:
    """ZeRO-3 units of a Llama (embedding, each decoder layer, final norm + head) as the
    coordinator stores them: frozen 16-bit weights above the persistence threshold (norms are
    persistent), LoRA-adapted linears in [N, K + fold_kp] rows (the folded adapter tail),
    with the projections a W^T copy would cover."""
    H, Fd, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    D = cfg.head_dim
    q, kv = cfg.num_attention_heads * D, cfg.num_key_value_heads * D
    fold = fold_kp if lora_r in (16, 32, 64) else 0
    qkv_ad = any(t in lora_targets for t in ("q_proj", "k_proj", "v_proj"))
    o_ad = "o_proj" in lora_targets
    gu_ad = any(t in lora_targets for t in ("gate_proj", "up_proj"))
    dn_ad = "down_proj" in lora_targets
    lin = [("qkv", q + 2 * kv, H, qkv_ad), ("o", H, q, o_ad), ("gate_up", 2 * Fd, H, gu_ad),
           ("down", H, Fd, dn_ad)]
    layer = {"stored": sum(n * (k + (fold if ad else 0)) for _, n, k, ad in lin),
             "wt": sum(n * k for _, n, k, _ in lin), "linears": len(lin)}
    units = [{"name": "embed", "stored": V * H, "wt": 0}]
    units += [dict(layer, name=f"layer{i}") for i in range(cfg.num_hidden_layers)]
    # the LM head keeps a W^T too unless LUMEN_LMHEAD_WT=0 (configure_backward_layout; the
    # ZeRO-3 keep schedule transposes its gathered head like the projections)
    head_wt = V * H if os.environ.get("LUMEN_LMHEAD_WT", "1") != "0" else 0
    units.append({"name": "head", "stored": V * H, "wt": head_wt, "linears": 1})
    return units


def lora_numel(cfg, lora_r: int = 16, targets=("q_proj", "k_proj", "v_proj", "o_proj")) -> int:
    H, Fd = cfg.hidden_size, cfg.intermediate_size
    q, kv = cfg.num_attention_heads * cfg.head_dim, cfg.num_key_value_heads * cfg.head_dim
    dims = {"q_proj": (H, q), "k_proj": (H, kv), "v_proj": (H, kv), "o_proj": (q, H),
            "gate_proj": (H, Fd), "up_proj": (H, Fd), "down_proj": (Fd, H)}
    return cfg.num_hidden_layers * sum(lora_r * (i + o) for t, (i, o) in dims.items()
                                       if t in targets)


def plan_zero3(cfg, world: int, hbm_bytes: float, tokens: int, checkpointing="auto",
               lora_r: int = 16, lora_targets=("q_proj", "k_proj", "v_proj", "o_proj"),
               elem_bytes: int = 2, align: int = 64) -> Dict:
    """The decisions a ZeRO-3 (stage3_max_live_parameters "auto") + LoRA rank makes, in the
    order it makes them, and the planned peak HBM.  ``tokens``: tokens per micro-step;
    ``checkpointing``: "auto" (the trainer CLI default) or a fixed policy (bench.py: "none")."""
    from .zero3 import ParamCoordinator

    units = llama_units(cfg, lora_targets, lora_r)
    padded = [_round_up(u["stored"], world * align) for u in units]
    total = sum(padded)
    n_lora = lora_numel(cfg, lora_r, lora_targets)
    # adapters: fp32 params + grads (flat, every rank), master / m / v sharded over the ranks
    lora_state = n_lora * 8 + n_lora * 12 / max(world, 1)
    if world == 1:
        schedule, reason, max_live = "identity", "world size 1", total
        shards = total * elem_bytes
        gathered = 0.0
        free = hbm_bytes - RUNTIME_OVERHEAD - shards - lora_state
        # persistent weights: configure_backward_layout's greedy per-linear W^T under the reserve
        budget = max(0.0, free - activation_reserve(hbm_bytes, "LUMEN_BWD_WT_RESERVE_GB"))
        wt = 0.0
        # in module order, as configure_backward_layout walks them: each layer's q|k|v, o,
        # gate|up, down, then the LM head
        per_lin = []
        H, Fd = cfg.hidden_size, cfg.intermediate_size
        q = cfg.num_attention_heads * cfg.head_dim
        kv = cfg.num_key_value_heads * cfg.head_dim
        for u in units:
            if u["name"].startswith("layer") and u["wt"]:
                per_lin += [(q + 2 * kv) * H, H * q, 2 * Fd * H, H * Fd]
            elif u["name"] == "head" and u["wt"]:
                per_lin.append(u["wt"])
        for n in per_lin:
            need = n * elem_bytes
            if need <= budget:
                budget -= need
                wt += need
        pool = 0
    else:
        shards = total / world * elem_bytes
        free = hbm_bytes - RUNTIME_OVERHEAD - shards - lora_state
        max_live = live_budget_elems(free, hbm_bytes, elem_bytes)
        schedule, reason = ParamCoordinator.auto_schedule(total, max_live, world, padded)
        mx = max(padded)
        if schedule == "keep":
            resident = [i for i, p in enumerate(padded) if p]
            pool = 0
        elif schedule == "hybrid":
            resident = ParamCoordinator.resident_plan(padded, max_live)
            rn = sum(padded[i] for i in resident)
            n_ring = sum(1 for i, p in enumerate(padded) if p and i not in resident)
            pool = max(2, min(int((max_live - rn) // mx), max(n_ring, 2)))
        else:
            resident = []
            pool = max(2, min(int(max_live // mx), len(padded)))
        gathered = (sum(padded[i] for i in resident) + pool * mx) * elem_bytes
        need_wt = sum(units[i]["wt"] for i in resident) * elem_bytes
        wt = need_wt if resident and transposes_fit(need_wt, gathered, free, hbm_bytes) else 0.0
    left = free - gathered - wt
    est = activation_bytes(cfg, tokens, "none")
    if checkpointing == "auto":
        policy = pick_checkpointing(est, left, selective_ok=not any(
            t in lora_targets for t in ("gate_proj", "up_proj", "down_proj")),
            n_layers=cfg.num_hidden_layers)
    else:
        policy = checkpointing
    act = activation_bytes(cfg, tokens, policy or "none")
    peak = RUNTIME_OVERHEAD + shards + lora_state + gathered + wt + act + TRANSIENT
    return {"model": cfg.name, "world": world, "hbm_gb": hbm_bytes / 1e9, "tokens": tokens,
            "schedule": schedule, "reason": reason, "max_live_elems": int(max_live),
            "total_elems": int(total), "ring_buffers": pool,
            "activation_reserve_gb": activation_reserve(hbm_bytes) / 1e9,
            "gb": {"runtime": RUNTIME_OVERHEAD / 1e9, "shards": shards / 1e9,
                   "lora_state": lora_state / 1e9, "gathered": gathered / 1e9,
                   "w_transposed": wt / 1e9, "activations": act / 1e9,
                   "transient": TRANSIENT / 1e9},
            "checkpointing": policy or "none", "activations_est_none_gb": est / 1e9,
            "peak_gb": peak / 1e9, "headroom": 1.0 - peak / hbm_bytes}


def main(argv=None) -> None:
    """``python -m lumen.parallel.memory_plan --model llama2-70b --world 8 --tokens 4096``"""
    import argparse
    import json

    from ..models import get_config

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-70b")
    ap.add_argument("--world", type=int, nargs="+", default=[8])
    ap.add_argument("--tokens", type=int, nargs="+", default=[4096])
    ap.add_argument("--hbm_gb", type=float, default=288.0)
    ap.add_argument("--checkpointing", nargs="+", default=["none", "auto"])
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    cfg = get_config(a.model)
    rows = [plan_zero3(cfg, w, a.hbm_gb * 1e9, t, c) for w in a.world for t in a.tokens
            for c in a.checkpointing]
    if a.json:
        print(json.dumps(rows, indent=1))
        return
    print("| world | tokens | ckpt (asked -> picked) | schedule | shards | gathered | W^T | "
          "activations | runtime+transient+LoRA | peak GB | headroom |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for r, c in zip(rows, [c for _ in a.world for _ in a.tokens for c in a.checkpointing]):
        g = r["gb"]
        print(f"| {r['world']} | {r['tokens']} | {c} -> {r['checkpointing']} | {r['schedule']} | "
              f"{g['shards']:.1f} | {g['gathered']:.1f} | {g['w_transposed']:.1f} | "
              f"{g['activations']:.1f} | {g['runtime'] + g['transient'] + g['lora_state']:.1f} | "
              f"{r['peak_gb']:.1f} | {100 * r['headroom']:.1f}% |")


if __name__ == "__main__":
    main()
