"""Custom IPC all-reduce (lumen/csrc/kernels/custom_ar.hip) on the GPU.

2, 4 or 8 processes share the box's one GPU: the IPC mapping, epoch barriers, one-shot and two-shot
paths, odd block counts, in-place / out-of-place and hipGraph replay are all exercised.  On a
shared device the peer loads stay on-chip, so this proves the protocol and numerics, not xGMI
bandwidth.  Every output must be bit-identical to the host f32 sum in rank order."""
import json
import socket

import pytest
import torch.multiprocessing as mp

from tests._dist_worker import car_gather_worker, car_worker

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_processes_one_gpu(world, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(car_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    res = json.loads((tmp_path / "car.json").read_text())
    bad = [c for c in res["cases"] if c["mismatches"]]
    assert not bad, bad
    assert len(res["cases"]) == 36
    assert res["graph_mismatches"] == 0
    assert res["err"] == 0
    print("custom all-reduce latency on a shared GPU (us):", res["timing_us"])


@pytest.mark.parametrize("world", [2, 8])
def test_custom_allgather_columns(world, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(car_gather_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    assert json.loads((tmp_path / "gather.json").read_text())["mismatches"] == 0


def test_tp2_serving_on_one_gpu_matches_single_process(tmp_path):
    """TP=2 engine + worker on the same GPU (bf16): custom all-reduce + graph-captured decode
    follow the un-sharded f32 model's greedy choice (teacher-forced, so one bf16 near-tie
    cannot derail the rest of a sequence)."""
    import torch

    from tests._dist_worker import _tp_test_model, serve_tp_gpu_worker

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(serve_tp_gpu_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    got = torch.load(tmp_path / "tp_gpu_out.pt", weights_only=True)
    info = got["info"]
    assert info["car"] and info["graphs"] and info["captured"], info
    assert info["car_calls"] > 0
    ref_model = _tp_test_model()
    prompts = [[5, 9, 33, 7], list(range(3, 30)), [42, 43]]
    agree, total = 0, 0
    for p, out in zip(prompts, got["out"]):
        assert len(out) == 8
        with torch.no_grad():
            logits = ref_model(torch.tensor(p + out)[None]).float().reshape(len(p) + 8, -1)
        pred = logits.argmax(-1)[len(p) - 1:len(p) - 1 + 8].tolist()
        assert pred[0] == out[0], (p, pred, out)
        agree += sum(int(a == b) for a, b in zip(pred, out))
        total += 8
    assert agree / total >= 0.85, (agree, total)


def test_custom_allreduce_peer_timeout_raises(tmp_path):
    """A peer that never arrives: the barrier deadline (2 s) ends the kernel, the pinned host
    error word is raised and ``poll()`` -- what the serving engine calls after each step --
    raises instead of returning a half-reduced tensor."""
    from tests._dist_worker import car_timeout_worker

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(car_timeout_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = json.loads((tmp_path / "car_timeout.json").read_text())
    assert res["first"] == 2.0
    assert res["raised"] is True and res["err_word"] == 1
