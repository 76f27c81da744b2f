"""TP serving greedy tokens on the box's one GPU under several carriers: TP=1, TP=W over RCCL
with / without the custom all-reduce (LUMEN_CUSTOM_AR), TP=W over gloo.  Prints each run's
tokens and which of them agree.

    python scripts/probes/tp_diag.py [--world 8] [--model tiny-llama-tp8]
"""
import argparse
import os
import socket
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(world, backend, model, env):
    from tests._dist_worker import serve_tp_gpu_worker

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        d = tempfile.mkdtemp()
        mp.start_processes(serve_tp_gpu_worker, args=(world, _port(), d, backend, model),
                           nprocs=world, join=True, start_method="spawn")
        return torch.load(os.path.join(d, "tp_gpu_out.pt"), weights_only=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="tiny-llama-tp8")
    a = ap.parse_args()
    runs = {"tp1": run(1, "nccl", a.model, {})}
    for name, be, env in (("nccl_car", "nccl", {}), ("nccl_nocar", "nccl", {"LUMEN_CUSTOM_AR": "0"}),
                          ("gloo_car", "gloo", {}), ("gloo_nocar", "gloo", {"LUMEN_CUSTOM_AR": "0"})):
        try:
            runs[name] = run(a.world, be, a.model, env)
        except Exception as e:  # noqa: BLE001
            print(name, "ERROR", repr(e)[:300], flush=True)
    for k, r in runs.items():
        print(k, r["out"], {x: r["info"].get(x) for x in ("car", "graphs", "car_calls")}, flush=True)
    base = runs["tp1"]["out"]
    for k, r in runs.items():
        print("agree_with_tp1", k, [x == y for x, y in zip(r["out"], base)], flush=True)


if __name__ == "__main__":
    main()
