"""World-size-portable ZeRO checkpoints: resharding and fp32 consolidation.

Reference behaviour: resume goes through HF Trainer / DeepSpeed (training/train_deepspeed_zero2.py:
302-332) whose ZeRO checkpoints ship ``zero_to_fp32.py`` (SURVEY 2.7 checkpoint layout), so a
run can be consolidated or resumed on a different number of GPUs.

lumen's optimizer state is ONE flat f32 buffer (``FlatTrainable``) cut into buckets; bucket b is
padded to a multiple of ``world * 64`` and split evenly over ranks, and a rank's shard is the
concatenation of its slice of every bucket.  Padding therefore depends on the world size, so a
shard is not portable by itself.  Every shard file carries the layout (world size, bucket
offsets / sizes, per-parameter flat offsets) and resharding is, per bucket, concatenate the old
slices -> read each parameter's range by name -> write it into the new layout -> take this
rank's new slices.  Parameters are matched by name, so bucket-size changes are fine too.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, List, Optional

import torch

_SHARD_RE = re.compile(r"zero_pp_rank_(\d+)_mp_rank_00_optim_states\.pt$")
STATE_KEYS = ("master", "exp_avg", "exp_avg_sq")


def shard_file(tag_dir: str, rank: int) -> str:
    return os.path.join(tag_dir, f"zero_pp_rank_{rank}_mp_rank_00_optim_states.pt")


def engine_layout(engine) -> Dict:
    """Layout of the engine's flat trainable buffer (plain Python values: weights_only-safe)."""
    names = {id(p): n for n, p in engine.model.named_parameters()}
    params = []
    for b in engine.flat.buckets:
        o = b.off
        for p in b.params:
            params.append((names[id(p)], o, p.numel()))
            o += p.numel()
    return {"world": engine.env.world_size, "sharded": bool(engine.sharded),
            "buckets": [(b.off, b.size) for b in engine.flat.buckets],
            "params": params, "numel": engine.flat.numel}


def _same_layout(a: Dict, b: Dict) -> bool:
    return all(a.get(k) == b.get(k) for k in ("world", "sharded", "buckets", "params"))


def _full_from_shards(shards: List[Dict], layout: Dict, key: str) -> torch.Tensor:
    """Reassemble the full flat buffer of ``key`` from every old rank's shard."""
    if not layout["sharded"]:
        return shards[0]["optimizer"][key].float()
    W = layout["world"]
    full = torch.zeros(layout["numel"], dtype=torch.float32)
    for r, sd in enumerate(shards):
        src = sd["optimizer"][key]
        so = 0
        for off, size in layout["buckets"]:
            s = size // W
            full[off + r * s:off + (r + 1) * s] = src[so:so + s]
            so += s
    return full


def read_shards(tag_dir: str) -> List[Dict]:
    files = {}
    for f in glob.glob(os.path.join(tag_dir, "zero_pp_rank_*_mp_rank_00_optim_states.pt")):
        m = _SHARD_RE.search(f)
        if m:
            files[int(m.group(1))] = f
    if not files:
        raise FileNotFoundError(f"no ZeRO shard files in {tag_dir}")
    first = torch.load(files[min(files)], map_location="cpu", weights_only=True)
    layout = first.get("layout")
    if layout is None:
        raise ValueError(f"{tag_dir}: shards carry no layout (saved before resharding support)")
    W = layout["world"]
    missing = [r for r in range(W) if r not in files]
    if missing:
        raise FileNotFoundError(f"{tag_dir}: shard files of ranks {missing} are missing")
    return [first] + [torch.load(files[r], map_location="cpu", weights_only=True)
                      for r in range(1, W)]


def consolidate(tag_dir: str) -> Dict[str, Dict[str, torch.Tensor]]:
    """{param name: {master, exp_avg, exp_avg_sq}} f32 full tensors (flat, 1-D)."""
    shards = read_shards(tag_dir)
    layout = shards[0]["layout"]
    fulls = {k: _full_from_shards(shards, layout, k) for k in STATE_KEYS}
    return {name: {k: fulls[k][o:o + n].clone() for k in STATE_KEYS}
            for name, o, n in layout["params"]}


def reshard_state(tag_dir: str, engine, rank: int) -> Dict:
    """State dict for ``engine`` (this rank) built from a checkpoint of any world size."""
    shards = read_shards(tag_dir)
    old = shards[0]["layout"]
    new = engine_layout(engine)
    fulls = {k: _full_from_shards(shards, old, k) for k in STATE_KEYS}
    where = {name: (o, n) for name, o, n in old["params"]}
    new_full = {k: torch.zeros(new["numel"], dtype=torch.float32) for k in STATE_KEYS}
    for name, o, n in new["params"]:
        if name not in where:
            raise KeyError(f"parameter {name} is not in the checkpoint {tag_dir}")
        oo, on = where[name]
        if on != n:
            raise ValueError(f"{name}: {on} elements in the checkpoint, {n} in the model")
        for k in STATE_KEYS:
            new_full[k][o:o + n] = fulls[k][oo:oo + on]
    if new["sharded"]:
        W = new["world"]
        opt = {k: torch.cat([v[off + rank * (size // W):off + (rank + 1) * (size // W)]
                             for off, size in new["buckets"]]) for k, v in new_full.items()}
    else:
        opt = new_full
    src = shards[0]
    o = dict(src["optimizer"])
    o.update(opt)
    sd = dict(src)
    sd["optimizer"] = o
    sd["world_size"] = new["world"]
    sd["shard_numel"] = opt["master"].numel()
    sd["layout"] = new
    return sd


def load_engine_state(tag_dir: str, engine, rank: int) -> None:
    """Load this rank's optimizer shard; reshard when the world size / layout changed."""
    f = shard_file(tag_dir, rank)
    sd: Optional[Dict] = None
    if os.path.exists(f):
        sd = torch.load(f, map_location="cpu", weights_only=True)
        lay = sd.get("layout")
        if lay is None and sd["shard_numel"] == engine.opt.master.numel() and \
                sd.get("world_size") == engine.env.world_size:
            engine.load_state_dict(sd)   # pre-layout checkpoint, same world
            return
        if lay is not None and _same_layout(lay, engine_layout(engine)):
            engine.load_state_dict(sd)
            return
    engine.load_state_dict(reshard_state(tag_dir, engine, rank))
