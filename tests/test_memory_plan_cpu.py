"""HBM plan of ZeRO-3 + LoRA (lumen/parallel/memory_plan.py) -- the decisions the runtime makes
from free HBM (live budget -> schedule, W^T copies, activation recompute), replayed for a model,
world size and device capacity without allocating.  BASELINE config 5: Llama-2-70B ZeRO-3 + LoRA
on 8 x MI355X (288 GB each)."""
import pytest

from lumen.models import get_config
from lumen.parallel.memory_plan import (activation_reserve, live_budget_elems, llama_units,
                                        lora_numel, plan_zero3)
from lumen.parallel.zero3 import ParamCoordinator

HBM = 288e9


def test_llama70b_world8_plan_keeps_one_copy_with_headroom():
    cfg = get_config("llama2-70b")
    # bench.py's configuration (no recompute) at 8 x 512 and 4 x 512 tokens per micro-step, and
    # the trainer CLI default (--gradient_checkpointing auto) at 8 x 512
    for tokens, ck, want_ck in ((4096, "none", "none"), (2048, "none", "none"),
                                (4096, "auto", "selective")):
        p = plan_zero3(cfg, 8, HBM, tokens, ck)
        assert p["schedule"] == "keep", p            # one gathered copy, resident
        # auto recomputes only as many layers as the budget needs ("selective:N")
        assert p["checkpointing"].split(":")[0] == want_ck, p
        assert p["headroom"] >= 0.10, p               # >= 10% of the 288 GB left over
        # W^T of the 70B projections (129 GB) does not fit next to the gathered copy: the
        # backward runs the NN input-gradient GEMMs instead of over-committing HBM
        assert p["gb"]["w_transposed"] == 0.0
        assert p["gb"]["gathered"] == pytest.approx(2 * p["total_elems"] / 1e9)
        assert p["gb"]["shards"] == pytest.approx(p["gb"]["gathered"] / 8, rel=1e-6)
    # the trainable set: 65,536,000 adapters (tests/test_lora_peft.py)
    assert lora_numel(cfg) == 65_536_000


def test_schedule_moves_with_world_and_budget():
    cfg70, cfg7 = get_config("llama2-70b"), get_config("llama2-7b")
    assert plan_zero3(cfg70, 1, HBM, 2048, "none")["schedule"] == "identity"
    for w in (2, 4, 8):
        assert plan_zero3(cfg70, w, HBM, 2048, "auto")["schedule"] == "keep"
        p7 = plan_zero3(cfg7, w, HBM, 4096, "none")
        assert p7["schedule"] == "keep" and p7["gb"]["w_transposed"] > 0   # 7B: W^T fits too
    # a smaller device: 70B at world 2 on 192 GB no longer holds a copy -> hybrid ring
    p = plan_zero3(cfg70, 2, 192e9, 2048, "auto")
    assert p["schedule"] in ("hybrid", "release") and p["ring_buffers"] >= 2
    assert p["headroom"] > 0


def test_plan_tracks_measured_single_gpu_peaks():
    """World-1 plans against the measured max_memory_allocated of bench.py runs (the plan adds
    the runtime overhead that allocator counter does not see): Llama-2-7B 8 x 512 = 40.9 GB
    (BENCH_r04.json), Llama-2-70B 4 x 512 = 265.7 GB (profiles/r4_70b)."""
    for name, tokens, measured in (("llama2-7b", 4096, 40.9), ("llama2-70b", 2048, 265.7)):
        p = plan_zero3(get_config(name), 1, HBM, tokens, "none")
        alloc = p["peak_gb"] - p["gb"]["runtime"]
        assert abs(alloc - measured) / measured < 0.15, (name, alloc, measured, p["gb"])


def test_runtime_budget_helpers_are_the_planners():
    """The coordinator's "auto" live budget and schedule come from the same helpers."""
    total = 288e9
    assert activation_reserve(total) == pytest.approx(0.25 * total)
    assert activation_reserve(100e9) == 48 * 2**30
    free = 250e9
    assert live_budget_elems(free, total, 2) == int((free - 0.25 * total) // 2)
    units = [u["stored"] for u in llama_units(get_config("llama2-70b"))]
    s, _ = ParamCoordinator.auto_schedule(sum(units), live_budget_elems(free, total, 2), 8, units)
    assert s == "keep"


def test_partial_recompute_picks_fewest_layers():
    """``auto`` with per-layer granularity: the fewest recomputed layers whose activations fit
    twice; selective before full; all layers -> the plain policy name."""
    from lumen.parallel.memory_plan import (SELECTIVE_FRACTION, activation_bytes,
                                            pick_checkpointing)

    L, est = 32, 100.0
    assert pick_checkpointing(est, 200, True, L) is False
    pol = pick_checkpointing(est, 150, True, L)
    k = int(pol.split(":")[1])
    frac = lambda k: 1 - k * (1 - SELECTIVE_FRACTION) / L  # noqa: E731
    assert pol.startswith("selective:") and 2 * est * frac(k) <= 150 < 2 * est * frac(k - 1)
    assert pick_checkpointing(est, 2 * SELECTIVE_FRACTION * est, True, L) == "selective"
    assert pick_checkpointing(est, 110, True, L).startswith("full:")   # selective cannot fit
    assert pick_checkpointing(est, 150, False, L).startswith("full:")  # MLP not eligible
    assert pick_checkpointing(est, 1, True, L) == "full"
    assert pick_checkpointing(est, 150, True) == "selective"           # no granularity: as before
    assert pick_checkpointing(est, 110, True) == "full"
    cfg = get_config("llama2-7b")
    none = activation_bytes(cfg, 4096, "none")
    assert activation_bytes(cfg, 4096, "selective:16") == pytest.approx(
        none * (1 - 16 * (1 - SELECTIVE_FRACTION) / 32))
    assert activation_bytes(cfg, 4096, "selective:32") == activation_bytes(cfg, 4096, "selective")
    assert activation_bytes(cfg, 4096, "full:32") == pytest.approx(activation_bytes(cfg, 4096, "full"))


def test_lm_head_transpose_is_planned(monkeypatch):
    """The LM head's W^T (LUMEN_LMHEAD_WT, on by default) is in the plan: V * H elements on the
    head unit, and in the world-1 greedy W^T budget after the layers."""
    cfg = get_config("llama2-7b")
    V, H = cfg.vocab_size, cfg.hidden_size
    head = llama_units(cfg)[-1]
    assert head["name"] == "head" and head["wt"] == V * H
    with_head = plan_zero3(cfg, 1, HBM, 4096, "none")["gb"]["w_transposed"]
    monkeypatch.setenv("LUMEN_LMHEAD_WT", "0")
    assert llama_units(cfg)[-1]["wt"] == 0
    without = plan_zero3(cfg, 1, HBM, 4096, "none")["gb"]["w_transposed"]
    assert with_head - without == pytest.approx(V * H * 2 / 1e9)
