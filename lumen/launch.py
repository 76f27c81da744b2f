"""Process launcher: one rank per GPU, fail-fast.

    python -m lumen.launch --nproc_per_node 8 training/train_deepspeed_zero3.py --deepspeed ...
    python -m lumen.launch --num_gpus 4 ...            # deepspeed-launcher spelling
    srun python -m lumen.launch --nproc_per_node 8 ... # multi-node under SLURM

What the reference gets from the ``deepspeed`` runner / ``torchrun`` (training/train.ipynb:229-253,
700-703; training/train_deepspeed_zero1.py:9-12), rebuilt around its one failure
(training/train.ipynb:230,679,806 -- the runner widened a scheduler-restricted device set and a
rank died on an invalid ordinal):

* never widens visibility: ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` /
  ``CUDA_VISIBLE_DEVICES`` are honoured as given, and ``nproc_per_node`` larger than the visible
  device count is an error raised *before* any rank starts;
* sets ``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR``,
  ``MASTER_PORT`` (default 127.0.0.1:29500) and passes ``--local_rank=k`` like the deepspeed
  runner (disable with ``--no_local_rank_arg``);
* multi-node: ``--nnodes/--node_rank/--master_addr`` or the ``SLURM_*`` environment;
* fail-fast: when a rank exits non-zero the siblings get SIGTERM, then SIGKILL after a grace
  period, and the launcher exits with the first failing rank's code (training/train.ipynb:822-824);
* forwards SIGINT/SIGTERM to the ranks; optional per-rank log files (``--log_dir``).

The children are started as plain subprocesses of a launcher that never touches the GPU.
"""
from __future__ import annotations

import argparse
import glob
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional

_VIS_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _parse_visible(v: str) -> int:
    v = v.strip()
    if not v:
        return 0
    return len([x for x in v.split(",") if x.strip() != ""])


def visible_device_count(env: Optional[Dict[str, str]] = None) -> int:
    """Number of GPUs a child would see, without initialising any GPU runtime.

    The most restrictive of the *_VISIBLE_DEVICES variables wins; otherwise count the GPU
    agents in the KFD topology (CPU nodes report ``simd_count 0``)."""
    env = os.environ if env is None else env
    counts = [_parse_visible(env[k]) for k in _VIS_VARS if k in env]
    if counts:
        return min(counts)
    n = 0
    for props in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(props) as f:
                for line in f:
                    if line.startswith("simd_count") and int(line.split()[1]) > 0:
                        n += 1
                        break
        except OSError:
            continue
    return n


def _slurm_master_addr(env) -> Optional[str]:
    nodelist = env.get("SLURM_JOB_NODELIST") or env.get("SLURM_NODELIST")
    if not nodelist:
        return None
    try:
        out = subprocess.run(["scontrol", "show", "hostnames", nodelist], capture_output=True,
                             text=True, timeout=10)
        if out.returncode == 0 and out.stdout.strip():
            return out.stdout.split()[0]
    except (OSError, subprocess.TimeoutExpired):
        pass
    # fallback: "node[01-04],other" -> "node01"
    first = nodelist.split(",")[0]
    if "[" in first:
        pre, rng = first.split("[", 1)
        return pre + rng.rstrip("]").split(",")[0].split("-")[0]
    return first


def parse_args(argv: Optional[List[str]] = None):
    p = argparse.ArgumentParser(prog="python -m lumen.launch",
                                description="Launch one process per GPU (fail-fast)")
    p.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=None)
    p.add_argument("--num_gpus", "--num-gpus", type=int, default=None,
                   help="deepspeed-runner spelling of --nproc_per_node")
    p.add_argument("--nnodes", type=int, default=None)
    p.add_argument("--node_rank", "--node-rank", type=int, default=None)
    p.add_argument("--master_addr", "--master-addr", default=None)
    p.add_argument("--master_port", "--master-port", type=int, default=None)
    p.add_argument("--no_local_rank_arg", action="store_true",
                   help="do not append --local_rank=k to the script's arguments")
    p.add_argument("--log_dir", default=None, help="write rank k's output to log_dir/rank_k.log")
    p.add_argument("--grace", type=float, default=10.0,
                   help="seconds between SIGTERM and SIGKILL when tearing siblings down")
    p.add_argument("--module", "-m", action="store_true", help="run the target as a module")
    p.add_argument("script")
    p.add_argument("script_args", nargs=argparse.REMAINDER)
    return p.parse_args(argv)


def build_rank_envs(a, env: Optional[Dict[str, str]] = None) -> List[Dict[str, str]]:
    env = dict(os.environ if env is None else env)
    nproc = a.nproc_per_node or a.num_gpus
    vis = visible_device_count(env)
    if nproc is None:
        nproc = int(env.get("SLURM_GPUS_ON_NODE", 0)) or vis or 1
    # (LUMEN_SHARED_GPU_REHEARSAL=1: ranks deliberately share devices, lumen.parallel.dist)
    if vis > 0 and nproc > vis and env.get("LUMEN_SHARED_GPU_REHEARSAL") != "1":
        raise SystemExit(f"lumen.launch: {nproc} ranks per node requested but only {vis} GPU(s) "
                         f"are visible to this job; refusing to widen the device set")
    nnodes = a.nnodes or int(env.get("SLURM_NNODES", 1))
    node_rank = a.node_rank if a.node_rank is not None else int(env.get("SLURM_NODEID", 0))
    master = a.master_addr or env.get("MASTER_ADDR") or (
        _slurm_master_addr(env) if nnodes > 1 else None) or "127.0.0.1"
    port = a.master_port or int(env.get("MASTER_PORT", 29500))
    world = nnodes * nproc
    envs = []
    for lr in range(nproc):
        e = dict(env)
        e.update(RANK=str(node_rank * nproc + lr), LOCAL_RANK=str(lr), WORLD_SIZE=str(world),
                 LOCAL_WORLD_SIZE=str(nproc), GROUP_RANK=str(node_rank), MASTER_ADDR=master,
                 MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL peer buffers
        envs.append(e)
    return envs


def build_cmd(a, local_rank: int) -> List[str]:
    cmd = [sys.executable, "-u"]
    cmd += ["-m", a.script] if a.module else [a.script]
    cmd += list(a.script_args)
    if not a.no_local_rank_arg:
        cmd.append(f"--local_rank={local_rank}")
    return cmd


def _terminate(procs, grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            try:
                p.kill()
            except ProcessLookupError:
                pass
            p.wait()


def launch(a) -> int:
    envs = build_rank_envs(a)
    procs: List[subprocess.Popen] = []
    files = []
    if a.log_dir:
        os.makedirs(a.log_dir, exist_ok=True)
    for lr, e in enumerate(envs):
        out = None
        if a.log_dir:
            out = open(os.path.join(a.log_dir, f"rank_{e['RANK']}.log"), "w")
            files.append(out)
        procs.append(subprocess.Popen(build_cmd(a, lr), env=e, stdout=out,
                                      stderr=subprocess.STDOUT if out else None))

    def _forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    old = {s: signal.signal(s, _forward) for s in (signal.SIGINT, signal.SIGTERM)}
    rc = 0
    try:
        alive = set(range(len(procs)))
        while alive:
            for i in list(alive):
                code = procs[i].poll()
                if code is None:
                    continue
                alive.discard(i)
                if code != 0:
                    print(f"lumen.launch: rank {envs[i]['RANK']} exited with code {code}; "
                          f"stopping {len(alive)} sibling rank(s)", file=sys.stderr, flush=True)
                    rc = code if code > 0 else 128 - code
                    _terminate([procs[j] for j in alive], a.grace)
                    alive.clear()
                    break
            time.sleep(0.1)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
        for f in files:
            f.close()
    return rc


def main(argv: Optional[List[str]] = None) -> int:
    return launch(parse_args(argv))


if __name__ == "__main__":
    sys.exit(main())
