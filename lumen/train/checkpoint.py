"""Checkpoint / resume.

Reference behaviour: HF Trainer + DeepSpeed periodic checkpoints ``{output_dir}/checkpoint-{N}``
every ``save_steps`` (100) with ``save_total_limit`` rotation (training/train_deepspeed_zero1.py:
242-245), discovery of the newest ``checkpoint-<N>`` for ``--resume_from_checkpoint``
(training/train_deepspeed_zero1.py:266-279) and a final PEFT export (train_baseline.py:226-228).
The HF/DeepSpeed layout holds the adapter, ``trainer_state.json``, per-rank RNG state and a
``global_step{N}/`` dir of ZeRO shards + ``latest``.

lumen writes the same directory shape with its own shard format:
    checkpoint-N/adapter_config.json, adapter_model.safetensors     (rank 0, PEFT format)
    checkpoint-N/trainer_state.json                                 (rank 0)
    checkpoint-N/rng_state_{rank}.pth                               (every rank)
    checkpoint-N/global_stepN/zero_pp_rank_{r}_mp_rank_00_optim_states.pt  (every rank: f32
        master / exp_avg / exp_avg_sq shard + step + loss-scaler state; tensors and plain
        Python values only, so it loads with ``torch.load(weights_only=True)``)
    checkpoint-N/latest                                             ("global_stepN")
Resume is resolved on EVERY rank (fixes reference quirk 7: rank-0-only discovery).

``AsyncCheckpointer`` snapshots the state to host memory on the training
thread and writes the files on a side thread; ranks signal completion with marker files, and
rank 0 writes ``trainer_state.json`` -- the completeness marker ``latest_checkpoint`` looks
for -- only after every rank's shard is on disk, so a crash mid-save never yields a checkpoint
that resume would pick.  Every save carries a nonce (broadcast from rank 0 on the training
thread): a marker counts only if it holds the current nonce, and rank 0 removes a re-saved
directory's old ``trainer_state.json`` / ``latest`` before any rank writes, so stale markers of
a crashed earlier save at the same step can never complete a half-written checkpoint.  No
collective runs off the training thread.

World-size portability: every shard file carries the flat-buffer layout (bucket offsets, per-
parameter offsets, world size), so ``load_checkpoint`` reshards a checkpoint saved at world N
into world M (``lumen.train.reshard``), and ``scripts/zero_to_fp32.py`` consolidates the f32
master weights (DeepSpeed's ``zero_to_fp32.py`` equivalent).
"""
from __future__ import annotations

import json
import os
import re
import shutil
import threading
import time
from typing import Dict, Optional

import torch

from ..lora import adapter_state_dict, load_adapter, save_adapter
from ..parallel.dist import barrier

_CKPT_RE = re.compile(r"^checkpoint-(\d+)$")


def list_checkpoints(output_dir: str):
    if not os.path.isdir(output_dir):
        return []
    out = []
    for d in os.listdir(output_dir):
        m = _CKPT_RE.match(d)
        if m and os.path.isdir(os.path.join(output_dir, d)):
            out.append((int(m.group(1)), os.path.join(output_dir, d)))
    return sorted(out)


def latest_checkpoint(output_dir: str) -> Optional[str]:
    """Newest *complete* checkpoint-<N> (trainer_state.json present)."""
    for step, path in reversed(list_checkpoints(output_dir)):
        if os.path.exists(os.path.join(path, "trainer_state.json")):
            return path
    return None


def _rng_state():
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def save_checkpoint(output_dir: str, engine, model, trainer_state: Dict, env,
                    save_total_limit: Optional[int] = None, base_model_name: str = "") -> str:
    step = engine.global_step
    path = os.path.join(output_dir, f"checkpoint-{step}")
    os.makedirs(path, exist_ok=True)
    gs = os.path.join(path, f"global_step{step}")
    os.makedirs(gs, exist_ok=True)
    sd = engine.state_dict()
    torch.save(sd, os.path.join(gs, f"zero_pp_rank_{env.rank}_mp_rank_00_optim_states.pt"))
    torch.save(_rng_state(), os.path.join(path, f"rng_state_{env.rank}.pth"))
    barrier()
    if env.rank == 0:
        save_adapter(model, path, base_model_name)
        with open(os.path.join(path, "latest"), "w") as f:
            f.write(f"global_step{step}")
        with open(os.path.join(path, "trainer_state.json"), "w") as f:
            json.dump(trainer_state, f, indent=2)
        if save_total_limit:
            ckpts = list_checkpoints(output_dir)
            for _, old in ckpts[:-save_total_limit]:
                shutil.rmtree(old, ignore_errors=True)
    barrier()
    return path


def load_checkpoint(path: str, engine, model, env) -> Dict:
    with open(os.path.join(path, "latest")) as f:
        tag = f.read().strip()
    load_adapter(model, path, apply=False)
    from .reshard import load_engine_state

    load_engine_state(os.path.join(path, tag), engine, env.rank)
    rng = os.path.join(path, f"rng_state_{env.rank}.pth")
    if os.path.exists(rng):
        st = torch.load(rng, map_location="cpu", weights_only=True)
        torch.set_rng_state(st["cpu"])
        if "cuda" in st and torch.cuda.is_available():
            torch.cuda.set_rng_state(st["cuda"])
    else:
        # resumed at a larger world size: a rank with no saved state gets its own stream
        # (seeded from the checkpoint step and its rank), never a copy of another rank's --
        # copied states would draw the same LoRA-dropout masks on several ranks
        with open(os.path.join(path, "trainer_state.json")) as f:
            step = int(json.load(f).get("global_step", 0))
        seed = (step * 1_000_003 + 7919 * (env.rank + 1)) % (2**63)
        torch.manual_seed(seed)
    with open(os.path.join(path, "trainer_state.json")) as f:
        return json.load(f)


def _marker(gs: str, rank: int) -> Optional[str]:
    try:
        with open(os.path.join(gs, f".done_{rank}")) as f:
            return f.read()
    except OSError:
        return None


def _to_host(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    return obj


class AsyncCheckpointer:
    """Background checkpoint writer with the same on-disk layout as ``save_checkpoint``."""

    def __init__(self, timeout_s: float = 3600.0):
        self.thread: Optional[threading.Thread] = None
        self.error: Optional[BaseException] = None
        self.timeout_s = timeout_s

    def wait(self) -> None:
        if self.thread is not None:
            self.thread.join()
            self.thread = None
        if self.error is not None:
            err, self.error = self.error, None
            raise RuntimeError("asynchronous checkpoint save failed") from err

    def save(self, output_dir: str, engine, model, trainer_state: Dict, env,
             save_total_limit: Optional[int] = None, base_model_name: str = "") -> str:
        self.wait()  # one save in flight at a time
        step = engine.global_step
        path = os.path.join(output_dir, f"checkpoint-{step}")
        gs = os.path.join(path, f"global_step{step}")
        os.makedirs(gs, exist_ok=True)
        # invalidate a previous (possibly crashed) save into this directory BEFORE any rank
        # writes, then agree on this save's nonce (the collective orders the two)
        mine = os.path.join(gs, f".done_{env.rank}")
        if os.path.exists(mine):
            os.remove(mine)
        if env.rank == 0:
            for f in ("trainer_state.json", "latest"):
                if os.path.exists(os.path.join(path, f)):
                    os.remove(os.path.join(path, f))
        from ..parallel.dist import broadcast_object

        nonce = broadcast_object(f"{os.getpid()}-{time.time_ns()}-{step}" if env.rank == 0
                                 else None)
        sd = _to_host(engine.state_dict())        # device -> host snapshot on this thread
        rng = _rng_state()
        adapter = {k: v.to("cpu", copy=True) for k, v in adapter_state_dict(model).items()} \
            if env.rank == 0 else None
        state = json.loads(json.dumps(trainer_state))
        rank, world = env.rank, env.world_size

        def work():
            try:
                torch.save(sd, os.path.join(gs, f"zero_pp_rank_{rank}_mp_rank_00_optim_states.pt"))
                torch.save(rng, os.path.join(path, f"rng_state_{rank}.pth"))
                tmp = os.path.join(gs, f".done_{rank}.tmp")
                with open(tmp, "w") as f:
                    f.write(nonce)
                os.replace(tmp, os.path.join(gs, f".done_{rank}"))  # atomic: never half a nonce
                if rank != 0:
                    return
                deadline = time.time() + self.timeout_s
                while not all(_marker(gs, r) == nonce for r in range(world)):
                    if time.time() > deadline:
                        raise TimeoutError(f"ranks did not finish writing {path}")
                    time.sleep(0.05)
                save_adapter(model, path, base_model_name, state=adapter)
                with open(os.path.join(path, "latest"), "w") as f:
                    f.write(f"global_step{step}")
                with open(os.path.join(path, "trainer_state.json"), "w") as f:
                    json.dump(state, f, indent=2)
                for r in range(world):
                    os.remove(os.path.join(gs, f".done_{r}"))
                if save_total_limit:
                    done = [c for c in list_checkpoints(output_dir)
                            if os.path.exists(os.path.join(c[1], "trainer_state.json"))]
                    for _, old in done[:-save_total_limit]:
                        shutil.rmtree(old, ignore_errors=True)
            except BaseException as e:  # noqa: BLE001 - re-raised on the training thread
                self.error = e

        self.thread = threading.Thread(target=work, name=f"lumen-ckpt-{step}", daemon=True)
        self.thread.start()
        return path
