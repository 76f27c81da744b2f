"""ZeRO-0/1/2/3 on CPU/gloo (world_size 2) reproduce the single-process run (fp32).

Mirrors BASELINE.json config 1 ("LoRA ZeRO-1 on CPU/gloo world_size=2") and SURVEY 4's plan:
distributed correctness proven without a cluster.  Same global batch either way: world 2 x
micro 2 vs world 1 x micro 4; the sampler hands rank r samples r, r+W, ... so each step sees the
same samples.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tests._dist_worker import train_worker


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, stage, outdir, **kw):
    os.makedirs(outdir, exist_ok=True)
    port = _port()
    if world == 1:
        train_worker(0, 1, port, stage, outdir, **kw)
    else:
        mp.spawn(train_worker, args=(world, port, stage, outdir) + tuple(kw.values()),
                 nprocs=world, join=True)
    return torch.load(os.path.join(outdir, f"result_stage{stage}_w{world}.pt"), weights_only=True)


@pytest.fixture(scope="module")
def reference(tmp_path_factory):
    d = tmp_path_factory.mktemp("ref")
    return _run(1, 0, str(d), model="tiny-llama", micro=4, accum=1, steps=3)


def _close(a, b, tol=2e-5):
    assert a.keys() == b.keys()
    for k in a:
        assert torch.allclose(a[k], b[k], atol=tol, rtol=1e-4), (k, (a[k] - b[k]).abs().max())


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
def test_zero_stage_matches_single_process(stage, reference, tmp_path):
    r = _run(2, stage, str(tmp_path), model="tiny-llama", micro=2, accum=1, steps=3)
    assert len(r["losses"]) == len(reference["losses"]) == 3
    for a, b in zip(r["losses"], reference["losses"]):
        assert abs(a - b) < 1e-3
    _close(r["sd"], reference["sd"])
    # the adapters actually moved
    assert any(v.abs().sum() > 0 for k, v in r["sd"].items() if "lora_B" in k)


def test_zero3_release_mode_and_accumulation(tmp_path):
    """ZeRO-3 with a live-parameter budget below the model (units released after forward and
    re-gathered for backward) + gradient accumulation == single process."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama", micro=2, accum=2, steps=2)
    r = _run(2, 3, str(tmp_path / "b"), model="tiny-llama", micro=1, accum=2, steps=2,
             extra={"max_live": 1000})
    _close(r["sd"], ref["sd"])


@pytest.mark.parametrize("schedule,gc", [("keep", False), ("keep", True), ("release", True),
                                         ("release", "full"), ("keep", "selective")])
def test_zero3_schedules_accumulation_checkpointing(schedule, gc, tmp_path):
    """Every ZeRO-3 gather schedule (keep: gathered once, resident; release: a ring of buffers,
    every unit re-gathered at each use) with gradient accumulation, with and without
    activation checkpointing (True = the default selective policy; full per-layer recompute)
    == single process."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama", micro=2, accum=2, steps=2,
               extra={"fuse": False})
    r = _run(2, 3, str(tmp_path / "b"), model="tiny-llama", micro=1, accum=2, steps=2,
             extra={"schedule": schedule, "gc": gc, "fuse": False})
    _close(r["sd"], ref["sd"])


@pytest.mark.parametrize("schedule", ["keep", "release"])
def test_zero3_world1_partitioned(schedule, tmp_path, monkeypatch):
    """LUMEN_ZERO3_SINGLE=1: the coordinator at world size 1 (local gathers) == stage 0."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama", micro=2, accum=2, steps=2)
    monkeypatch.setenv("LUMEN_ZERO3_POISON", "1")  # NaN-poisoned buffers: no stale reads
    r = _run(1, 3, str(tmp_path / "b"), model="tiny-llama", micro=2, accum=2, steps=2,
             extra={"schedule": schedule, "gc": True, "single": True})
    _close(r["sd"], ref["sd"])


def test_zero1_opt125m_style_world2(tmp_path):
    """BASELINE config 1 plumbing: OPT LoRA ZeRO-1 over gloo world_size=2 (tiny OPT)."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-opt", micro=4, accum=1, steps=2)
    r = _run(2, 1, str(tmp_path / "b"), model="tiny-opt", micro=2, accum=1, steps=2)
    _close(r["sd"], ref["sd"])


def test_zero2_cpu_offload_optimizer(tmp_path):
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama", micro=4, accum=1, steps=2)
    r = _run(2, 2, str(tmp_path / "b"), model="tiny-llama", micro=2, accum=1, steps=2,
             extra={"offload": True})
    # C++ AVX-512 AdamW vs torch AdamW: same math, different rounding order
    _close(r["sd"], ref["sd"], tol=3e-4)


# ---- world size 4: every ZeRO-3 schedule on split communicators -----------------------------

def _layer_numel(model="tiny-llama-deep"):
    from lumen.models import get_config

    c = get_config(model)
    H, D = c.hidden_size, c.head_dim
    return (H * (c.num_attention_heads + 2 * c.num_key_value_heads) * D
            + c.num_attention_heads * D * H + 3 * H * c.intermediate_size + 2 * H)


@pytest.fixture(scope="module")
def deep_reference(tmp_path_factory):
    d = tmp_path_factory.mktemp("deepref")
    return _run(1, 0, str(d), model="tiny-llama-deep", micro=4, accum=2, steps=2,
                extra={"fuse": False})


@pytest.mark.parametrize("case", [
    dict(schedule="keep"),
    dict(schedule="keep", gc=True),
    # release, ring of 2 buffers: depth 1, nothing kept across the fwd->bwd turn
    dict(schedule="release", live_units=2),
    # release, ring of 5: depth 2 (prefetch bucket = 2 layers), 2 units reused at the turn
    dict(schedule="release", live_units=5, prefetch_units=2, reuse_units=2, gc=True),
    # release, ring of 5, default reuse distance: the ring serves reuse first (3 units kept)
    dict(schedule="release", live_units=5, prefetch_units=2),
    # release + reuse distance 0: every unit gathered twice
    dict(schedule="release", live_units=5, prefetch_units=1, reuse=0),
    # offloaded (host) shards: H2D + gather issued off the compute stream
    dict(schedule="keep", offload_param=True),
    # hybrid (the auto choice for this budget): 2 of the 6 layers resident, the rest through a
    # 2-buffer ring
    dict(schedule="hybrid", live_units=4, gc=True),
])
def test_zero3_world4_split_groups(case, deep_reference, tmp_path):
    """World 4 over gloo: every schedule, on a separate weight-gather process group, with
    gradient accumulation (and checkpointing where marked) == single-process stage 0."""
    L = _layer_numel()
    # fuse=False: the two accumulation micro-steps run as two forward/backward passes (the
    # coordinator's per-micro-step hooks), not as one fused batch
    extra = {"schedule": case["schedule"], "gc": case.get("gc", False), "fuse": False}
    if case["schedule"] == "hybrid":
        extra.pop("schedule")  # picked by the auto rule from the budget
    if "live_units" in case:
        extra["max_live"] = int(case["live_units"] * L * 1.02)
    if "prefetch_units" in case:
        extra["prefetch"] = int(case["prefetch_units"] * L * 1.02)
    if "reuse" in case:
        extra["reuse"] = case["reuse"]
    if "reuse_units" in case:
        extra["reuse"] = int(2 * case["reuse_units"] * L * 1.1)
    if case.get("offload_param"):
        extra["offload_param"] = True
    r = _run(4, 3, str(tmp_path), model="tiny-llama-deep", micro=1, accum=2, steps=2,
             extra=extra)
    _close(r["sd"], deep_reference["sd"])
    z = r["zero3"]
    assert z["schedule"] == case["schedule"] and z["world"] == 4
    # release / hybrid re-gather on their own communicator; keep gathers once, on the default
    assert z["gather_group_separate"] == (case["schedule"] != "keep")
    assert z["pool_overflows"] == 0
    n_units = 8
    if case["schedule"] == "hybrid":
        assert z["resident_units"] == 2 and z["pool_size"] == 2 and z["turn_keep"] == 0
        # 2 steps x 2 micro-steps x (6 ring units forward + 4 ring layers backward) + the two
        # resident layers, once
        assert z["gathers"] == 2 * 2 * (6 + 4) + 2
    elif case["schedule"] == "release":
        assert z["pool_size"] == case["live_units"]
        if case.get("reuse") == 0:
            assert z["turn_keep"] == 0
            # 2 steps x 2 micro-steps x (8 fwd + 6 bwd: every layer re-gathered, the head is
            # consumed at the turn)
            assert z["gathers"] == 2 * 2 * (n_units + n_units - 2)
        elif case["live_units"] == 5:
            keep = 2 if "reuse_units" in case else 3
            assert z["turn_keep"] == keep
            assert z["depth"] == 4 - keep
            assert z["gathers"] == 2 * 2 * (n_units + n_units - 2 - keep)
    else:
        assert z["gathers"] == n_units  # keep: once per unit, then resident


@pytest.mark.parametrize("schedule", ["keep", "release", "hybrid"])
def test_zero3_world8_split_groups(schedule, tmp_path):
    """World 8 over gloo (the rank count of the headline 8-GPU run): the schedule on its own
    weight-gather communicator next to the gradient group == single-process stage 0."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama-deep", micro=8, accum=1, steps=2)
    extra = {"schedule": schedule}
    if schedule != "keep":
        extra["max_live"] = int(3 * _layer_numel() * 1.02)
    r = _run(8, 3, str(tmp_path / "b"), model="tiny-llama-deep", micro=1, accum=1, steps=2,
             extra=extra)
    _close(r["sd"], ref["sd"])
    z = r["zero3"]
    assert z["schedule"] == schedule and z["world"] == 8
    assert z["gather_group_separate"] == (schedule != "keep")
    if schedule == "hybrid":
        assert z["resident_units"] == 1
    assert z["pool_overflows"] == 0


def test_accumulation_fusion_agreed_across_ranks(tmp_path):
    """Gradient-accumulation fusion (k equal-n_valid micro-batches as one forward / backward) is
    decided for every rank at once: variable-length rows give groups that are fusable on one
    rank and not on the other, and a rank-local decision would then issue a different number of
    ZeRO-3 gathers / reduce-scatters than its peer (a hang).  Fused == unfused results."""
    L = _layer_numel()
    ex = {"min_len": 15, "max_live": int(3 * L * 1.02)}   # ring schedule: gathers per forward
    got = _run(2, 3, str(tmp_path / "f"), model="tiny-llama-deep", micro=1, accum=2, steps=8,
               extra=dict(ex, fuse=True))
    ref = _run(2, 3, str(tmp_path / "u"), model="tiny-llama-deep", micro=1, accum=2, steps=8,
               extra=dict(ex, fuse=False))
    f = got["fusion"]
    assert f["vetoed"] > 0 and f["fused"] + f["vetoed"] + f["unfused"] == 8, f
    assert got["zero3"]["schedule"] in ("release", "hybrid")
    _close(got["sd"], ref["sd"], tol=1e-5)
    for a, b in zip(got["losses"], ref["losses"]):
        assert abs(a - b) < 1e-5 * max(1.0, abs(b))


def test_zero3_world1_identity(tmp_path):
    """World size 1 without forced partitioning: the one-rank partition is the whole unit, the
    coordinator binds parameters to it once and never gathers; == stage 0."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama", micro=2, accum=2, steps=2)
    r = _run(1, 3, str(tmp_path / "b"), model="tiny-llama", micro=2, accum=2, steps=2)
    _close(r["sd"], ref["sd"], tol=0)
    assert r["zero3"]["schedule"] == "identity" and r["zero3"]["gathers"] == 0


# ---- checkpoint resharding across world sizes ------------------------------------------------

@pytest.mark.parametrize("stage,w_save,w_load", [(2, 2, 1), (1, 1, 2), (3, 2, 4), (2, 4, 2)])
def test_resume_at_different_world_size(stage, w_save, w_load, tmp_path):
    """Save at world N after 2 steps, resume at world M (same global batch of 4) to step 4:
    the adapters match an uninterrupted world-N run (optimizer shards resharded by name)."""
    gb = 4
    ref = _run(w_save, stage, str(tmp_path / "ref"), model="tiny-llama", micro=gb // w_save,
               accum=1, steps=4)
    ck = str(tmp_path / "ck")
    _run(w_save, stage, str(tmp_path / "a"), model="tiny-llama", micro=gb // w_save, accum=1,
         steps=2, extra={"save_steps": 2, "ckdir": ck})
    r = _run(w_load, stage, str(tmp_path / "b"), model="tiny-llama", micro=gb // w_load,
             accum=1, steps=4, extra={"save_steps": 100, "ckdir": ck, "resume": True})
    _close(r["sd"], ref["sd"], tol=3e-5)
    assert r["res"]["global_step"] == 4


def test_zero_to_fp32_consolidation(tmp_path):
    """scripts/zero_to_fp32.py: world-2 ZeRO-2 shards -> one f32 PEFT adapter equal to the
    trained adapters."""
    import subprocess
    import sys

    from safetensors.torch import load_file

    ck = str(tmp_path / "ck")
    r = _run(2, 2, str(tmp_path / "a"), model="tiny-llama", micro=2, accum=1, steps=2,
             extra={"save_steps": 2, "ckdir": ck})
    out = str(tmp_path / "fp32")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run([sys.executable, os.path.join(root, "scripts", "zero_to_fp32.py"),
                    os.path.join(ck, "checkpoint-2"), out], check=True, cwd=root)
    got = load_file(os.path.join(out, "adapter_model.safetensors"))
    assert got.keys() == r["sd"].keys()
    for k in got:
        assert got[k].dtype == torch.float32
        assert torch.equal(got[k], r["sd"][k]), k
    st = torch.load(os.path.join(out, "optimizer_fp32.pt"), weights_only=True)
    assert all(set(v) == {"exp_avg", "exp_avg_sq"} for v in st.values())


def test_zero3_auto_schedule_rule():
    """``stage3_max_live_parameters: "auto"``: release below the model size, otherwise keep
    (frozen weights gathered once and kept resident) at every world size."""
    from lumen.parallel.zero3 import ParamCoordinator as PC

    assert PC.auto_schedule(100, 99, 8)[0] == "release"
    for w in (2, 3, 4, 8):
        s, why = PC.auto_schedule(100, 100, w)
        assert s == "keep" and "resident" in why
    # hybrid between the two: embedding 5, 8 layers of 10, head 5 (model 90)
    sizes = [5] + [10] * 8 + [5]
    assert PC.auto_schedule(90, 89, 8, sizes)[0] == "hybrid"
    assert PC.auto_schedule(90, 29, 8, sizes)[0] == "release"   # ring of 2 + not one layer
    assert PC.auto_schedule(90, 30, 8, sizes)[0] == "hybrid"
    # residents spread evenly over the decoder layers (indices 1..8)
    assert PC.resident_plan(sizes, 30) == [5]
    assert PC.resident_plan(sizes, 60) == [2, 4, 6, 8]
    assert PC.resident_plan(sizes, 89) == [1, 3, 4, 5, 7, 8]
    assert PC.resident_plan(sizes, 1000) == list(range(1, 9))
