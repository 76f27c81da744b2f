"""Custom IPC all-reduce (lumen/csrc/kernels/custom_ar.hip) on the GPU.

Two processes share the box's one GPU: the IPC mapping, epoch barriers, one-shot and two-shot
paths, odd block counts, in-place / out-of-place and hipGraph replay are all exercised.  On a
shared device the peer loads stay on-chip, so this proves the protocol and numerics, not xGMI
bandwidth.  Every output must be bit-identical to the host f32 sum in rank order."""
import json
import socket

import pytest
import torch.multiprocessing as mp

from tests._dist_worker import car_worker

pytestmark = pytest.mark.gpu


def test_custom_allreduce_two_processes_one_gpu(tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(car_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = json.loads((tmp_path / "car.json").read_text())
    bad = [c for c in res["cases"] if c["mismatches"]]
    assert not bad, bad
    assert len(res["cases"]) == 36
    assert res["graph_mismatches"] == 0
    assert res["err"] == 0
    print("custom all-reduce latency on a shared GPU (us):", res["timing_us"])
