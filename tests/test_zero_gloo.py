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


@pytest.mark.parametrize("schedule,gc", [("keep", False), ("keep", True), ("pipelined", True),
                                         ("release", True)])
def test_zero3_schedules_accumulation_checkpointing(schedule, gc, tmp_path):
    """Every ZeRO-3 gather schedule (keep: re-gather after each unit's backward; pipelined:
    next micro-step gathered one step ahead into a second buffer; release) with gradient
    accumulation, with and without activation checkpointing == single process."""
    ref = _run(1, 0, str(tmp_path / "a"), model="tiny-llama", micro=2, accum=2, steps=2)
    r = _run(2, 3, str(tmp_path / "b"), model="tiny-llama", micro=1, accum=2, steps=2,
             extra={"schedule": schedule, "gc": gc})
    _close(r["sd"], ref["sd"])


@pytest.mark.parametrize("schedule", ["keep", "pipelined", "release"])
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
