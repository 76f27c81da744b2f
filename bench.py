#!/usr/bin/env python3
"""Headline benchmark: Llama-2-7B LoRA fine-tuning with ZeRO-3, bf16, on N MI355X GPUs.

Metric (BASELINE.json): "train tok/s Llama-2-7B ZeRO-3+LoRA at 1/2/4/8 GPUs" -- whole-job
tokens/s over exactly --steps optimizer steps after --warmup untimed steps, bracketed by a
barrier + device synchronisation on both sides, max time over ranks.

Config (reference training/train_deepspeed_zero3.py + configs/ds_config_zero3.json, MI355X
variant configs/ds_config_zero3_mi355x.json): Llama-2-7B architecture (random init: offline),
LoRA r=16 alpha=32 dropout=0.05 on q/k/v/o, AdamW lr 2e-4, grad clip 1.0, seq 512 synthetic
tokens, 8 sequences per GPU per optimizer step (reference: micro 2 x accum 4 = 8; default
here micro 8 x accum 1 -- same samples per step, one ZeRO-3 gather per unit per step).
Baseline: the reference's only published number, 3.12 samples/s x 512 tokens = 1,597 tok/s
(ZeRO-2, 1x V100, training/train.ipynb:442).

Usage: python bench.py [--gpus N --steps K --warmup W]   (N>1: under torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_START = time.time()

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOK_S = 3.12 * 512  # training/train.ipynb:442 (samples/s) x max_length 512
METRIC = "train tok/s Llama-2-7B ZeRO-3+LoRA at 1/2/4/8 GPUs; serve tok/s + p50 TTFT"


def run_serve_bench(args) -> dict:
    """Serving half of the metric, after the timed training region (training model freed).

    One LLMEngine (Llama-2-7B TP=1: continuous batching, hipGraph decode, async scheduling, bf16
    KV, greedy) with the scheduling of the vLLM version the reference pins (vllm==0.6.0,
    requirements.txt:18): chunked prefill off, prefill-only steps while prompts wait, then decode
    steps, max_num_batched_tokens = max(max_model_len, 2048) = 4096 for Llama-2's 4096 context.
    Measurements of the same 256-request burst (512 in / 128 out, all arriving at t=0):
      * ``http`` -> ``extra.serve``: the reference's declared path -- the OpenAI HTTP server
        (4 spawned API processes on one port, ``lumen serve --api-server-count 4``: one Python
        front-end saturates at 256 streams) streaming ``/v1/completions`` to the async load
        client (4 processes, Locust's distributed-worker layout; the Locust request shape);
      * ``engine`` -> ``extra.serve_engine``: the same engine driven in-process (no HTTP);
      * ``extra.serve_chunked``: in-process again with lumen's mixed-step policy (chunked
        prefill, 2048 tokens per step: inter-token latency bounded by one mixed step instead of
        the whole prefill backlog -- the itl_max_ms the prefill-first records show).
    A failure is reported in the record, never fatal to the training number already measured."""
    import gc
    import types

    import torch

    gc.collect()
    torch.cuda.empty_cache()
    from lumen.bench.serve_bench import bench_engine, bench_http, make_engine

    a = types.SimpleNamespace(
        model=args.serve_model or args.model, max_model_len=1024, max_num_seqs=256,
        max_batched_tokens=4096, prefill_boost=int(os.environ.get("LUMEN_PREFILL_BOOST", "1")),
        no_graphs=False, sync_scheduling=False, kv_cache_dtype="auto",
        scheduling_policy=os.environ.get("LUMEN_SERVE_POLICY", "prefill_first"),
        num_requests=256, concurrency=256, prompt_len=512, max_tokens=128, temperature=0.0,
        request_rate=None, api_servers=int(os.environ.get("LUMEN_API_SERVERS", "4")),
        client_procs=int(os.environ.get("LUMEN_CLIENT_PROCS", "4")))
    keep = ("output_tok_s", "ttft_p50_ms", "ttft_p99_ms", "itl_p50_ms", "itl_p99_ms",
            "itl_max_ms", "itl_mean_ms", "wall_s", "total_tok_s", "output_tokens", "preemptions",
            "steps", "setup_s", "ok", "errors", "http_section_s")
    conf = {"model": a.model, "tp": 1, "requests": a.num_requests, "prompt_len": a.prompt_len,
            "max_tokens": a.max_tokens, "max_num_batched_tokens": a.max_batched_tokens,
            "scheduling_policy": a.scheduling_policy,
            "prefill_boost": a.prefill_boost, "kv_cache_dtype": "bf16",
            "sampling": "greedy, ignore_eos", "arrival": "all at t=0"}
    t0 = time.time()
    try:
        eng = make_engine(a)
        r = bench_engine(a, eng)
    except Exception as e:  # noqa: BLE001 - keep the training result
        return {"error": repr(e)[:500]}, None, None, None
    e_out = {k: r[k] for k in keep if k in r}
    e_out["bench_s"] = round(time.time() - t0, 1)
    e_out["config"] = dict(conf, async_scheduling=r.get("async_scheduling"),
                           mode="in-process engine")
    t1 = time.time()
    try:
        h = bench_http(a, eng)
    except Exception as e:  # noqa: BLE001 - the engine-mode number stands
        eng.shutdown()
        return {"error": "http: " + repr(e)[:500], "engine_fallback": e_out}, e_out, None, None
    h_out = {k: h[k] for k in keep if k in h}
    h_out["bench_s"] = round(time.time() - t1, 1)
    h_out["vs_engine"] = round(h["output_tok_s"] / max(r["output_tok_s"], 1e-9), 3)
    h_out["config"] = dict(conf, concurrency=a.concurrency, api_servers=a.api_servers,
                           client_procs=a.client_procs,
                           mode="OpenAI HTTP API (/v1/completions, SSE) + async load client")
    c_out = None
    if a.scheduling_policy != "chunked":
        t2 = time.time()
        try:  # same engine (graphs captured): only the scheduler's policy and budget change
            eng.scheduler.cfg.policy = "chunked"
            eng.scheduler.cfg.max_num_batched_tokens = 2048
            ac = types.SimpleNamespace(**dict(vars(a), scheduling_policy="chunked",
                                              max_batched_tokens=2048))
            c = bench_engine(ac, eng)
            c_out = {k: c[k] for k in keep if k in c}
            c_out["bench_s"] = round(time.time() - t2, 1)
            c_out["config"] = dict(conf, scheduling_policy="chunked", max_num_batched_tokens=2048,
                                   mode="in-process engine")
        except Exception as e:  # noqa: BLE001
            c_out = {"error": repr(e)[:500]}
    # the same burst with vLLM's non-greedy sampler settings (temperature 0.8, top-p 0.95,
    # top-k 50: the radix-select top-k / top-p kernel, kernels/sampling.hip), prefill-first
    s_out = None
    t3 = time.time()
    try:
        eng.scheduler.cfg.policy = "prefill_first"
        eng.scheduler.cfg.max_num_batched_tokens = a.max_batched_tokens
        asm = types.SimpleNamespace(**dict(vars(a), temperature=0.8, top_p=0.95, top_k=50))
        sm = bench_engine(asm, eng)
        s_out = {k: sm[k] for k in keep if k in sm}
        s_out["bench_s"] = round(time.time() - t3, 1)
        s_out["vs_greedy_engine"] = round(sm["output_tok_s"] / max(r["output_tok_s"], 1e-9), 3)
        s_out["config"] = dict(conf, sampling="temperature 0.8, top_p 0.95, top_k 50, ignore_eos",
                               mode="in-process engine")
    except Exception as e:  # noqa: BLE001
        s_out = {"error": repr(e)[:500]}
    eng.shutdown()
    return h_out, e_out, c_out, s_out


def run_serve_tp(args, env) -> dict:
    """TP = world serving after the training sections (N > 1): Llama-2-7B sharded over the N
    GPUs -- heads / FFN columns / vocab split, row-parallel sums on the custom IPC all-reduce
    (kernels/custom_ar.hip) over xGMI, decode buckets as hipGraphs, each step's host header over
    a gloo group and its payload as one RCCL broadcast (lumen/serve/tp.py).  Rank 0 drives the
    engine through the same 256-request burst as the TP = 1 section (engine mode, vLLM 0.6.0
    scheduling); the other ranks run the worker loop.  Returns rank 0's record (None elsewhere)."""
    import gc
    import types

    import torch

    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    from lumen.bench.serve_bench import bench_engine, make_engine
    from lumen.serve.tp import worker_loop

    nreq, plen, mtok = (int(x) for x in args.serve_tp_shape.split(","))
    a = types.SimpleNamespace(
        model=args.serve_model or args.model, max_model_len=1024, max_num_seqs=256,
        max_batched_tokens=4096, prefill_boost=1, no_graphs=False, sync_scheduling=False,
        kv_cache_dtype="auto", scheduling_policy="prefill_first", tp=env.world_size,
        num_requests=nreq, concurrency=nreq, prompt_len=plen, max_tokens=mtok, temperature=0.0,
        request_rate=None)
    t0 = time.time()
    eng = make_engine(a)
    if env.rank != 0:
        worker_loop(eng.runner)
        return None
    try:
        r = bench_engine(a, eng)
    finally:
        eng.shutdown()  # releases the workers' loops
    keep = ("output_tok_s", "ttft_p50_ms", "ttft_p99_ms", "itl_p50_ms", "itl_p99_ms",
            "itl_max_ms", "wall_s", "total_tok_s", "output_tokens", "steps", "graphs")
    out = {k: r[k] for k in keep if k in r}
    out["bench_s"] = round(time.time() - t0, 1)
    out["config"] = {"model": a.model, "tp": env.world_size, "requests": a.num_requests,
                     "prompt_len": a.prompt_len, "max_tokens": a.max_tokens,
                     "scheduling_policy": a.scheduling_policy,
                     "max_num_batched_tokens": a.max_batched_tokens, "kv_cache_dtype": "bf16",
                     "custom_allreduce": eng.runner.car is not None, "mode": "in-process engine"}
    car = eng.runner.car
    if car is not None and car.calibration is not None:
        # the crossovers measured on this TP group at engine start (replaces guessed limits)
        out["car_plan"] = car.calibration
    return out


def run_partitioned(args, env, ds_base, batches, schedule: str, max_live: float,
                    steps: int = 5, warmup: int = 2) -> dict:
    """Extra timed steps of a PARTITIONED ZeRO-3 schedule on a fresh model + engine (after the
    headline engine is freed): ``release`` / ``hybrid`` re-gather frozen weights every use over
    the weight-gather communicator -- the per-step xGMI traffic ``keep`` avoids.  At world size
    1 the partitioning is forced (LUMEN_ZERO3_SINGLE: every gather is a device copy)."""
    import copy
    import gc

    import torch
    import torch.distributed as dist

    from lumen.lora import LoraConfig, apply_lora
    from lumen.models import build_model
    from lumen.train.engine import ZeroEngine

    on_gpu = env.device.type == "cuda"
    gc.collect()
    if on_gpu:
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
    ds = copy.copy(ds_base)
    ds.stage3_max_live_parameters = int(max_live)
    saved = {k: os.environ.get(k) for k in ("LUMEN_ZERO3_SCHEDULE", "LUMEN_ZERO3_SINGLE")}
    os.environ["LUMEN_ZERO3_SCHEDULE"] = schedule
    if env.world_size == 1:
        os.environ["LUMEN_ZERO3_SINGLE"] = "1"
    try:
        torch.manual_seed(1234)
        model = build_model(args.model, dtype=ds.torch_dtype, device=env.device, init="random",
                            seed=0)
        apply_lora(model, LoraConfig(r=args.lora_r, lora_dropout=0.05))
        model.train()
        eng = ZeroEngine(model, ds, env)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    co = eng.coordinator

    def run(n, off):
        for s in range(n):
            for a in range(ds.grad_accum):
                b = batches[(off + s * ds.grad_accum + a) % len(batches)]
                loss = eng.forward(b)
                eng.backward(loss)
                eng.step()
        return loss

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
        if dist.is_initialized():
            from lumen.parallel.dist import barrier

            barrier()
            if on_gpu:
                torch.cuda.synchronize()

    run(warmup, 0)
    sync()
    gb0 = co.gathered_bytes
    co.pop_exposed_wait_ms()
    co.track_waits = True
    sk0 = eng.skipped_steps
    t1 = time.perf_counter()
    run(steps, warmup)
    sync()
    dt = time.perf_counter() - t1
    exposed = co.pop_exposed_wait_ms()
    t = torch.tensor([dt, exposed, torch.cuda.max_memory_allocated() / 1e9 if on_gpu else 0.0],
                     dtype=torch.float32 if on_gpu else torch.float64, device=env.device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, exposed, peak = (float(x) for x in t.tolist())
    st = co.stats()
    out = {"schedule": st["schedule"], "stage3_max_live_parameters": int(max_live),
           "resident_units": st["resident_units"], "units": st["units"],
           "ring_buffers": st["pool_size"], "turn_keep": st["turn_keep"],
           "steps": steps, "warmup": warmup,
           "ms_per_step": round(dt / steps * 1000, 2),
           "tok_s": round(env.world_size * ds.micro_batch * ds.grad_accum * args.seq_len
                          * steps / dt, 1),
           "peak_hbm_gb_max_rank": round(peak, 2),
           "gathered_mb_per_step": round((co.gathered_bytes - gb0) / 1e6 / steps, 1),
           "exposed_gather_wait_ms_per_step_max_rank": round(exposed / steps, 2),
           "skipped_nonfinite": eng.skipped_steps - sk0,
           "forced_world1": env.world_size == 1}
    eng.close()
    del eng, model, co
    gc.collect()
    if on_gpu:
        torch.cuda.empty_cache()
    return out


def run_comm_probe(env, gather_group=None, unit_mb: float = 386.0, bucket_numel: int = 2_000_000,
                   car_sizes=(8 << 10, 256 << 10, 2 << 20), iters: int = 5) -> dict:
    """N > 1: what the transport itself delivers, so a sub-linear scaling record says whether
    the links or the schedule are at fault (Next #4).  Collective on every rank.

    * ``all_gather``: one Llama-2-7B decoder unit (386 MiB of bf16) gathered with
      ``all_gather_into_tensor`` on the weight-gather communicator (the default group when the
      schedule has none) -- time, algorithm GB/s (bytes / time) and bus GB/s (x (W-1)/W, the
      nccl-tests convention: the per-rank link load a ring or mesh must carry);
    * ``reduce_scatter``: one LoRA gradient bucket (2e6 fp32 elements);
    * ``allreduce``: custom one-shot / two-shot vs RCCL all-reduce latency at the TP decode
      message sizes (GPU only: the IPC kernel needs the native extension).
    Times are the max over ranks of the mean over ``iters`` calls after one warm-up call."""
    import torch
    import torch.distributed as dist

    W = env.world_size
    on_gpu = env.device.type == "cuda"
    dev = env.device
    res = {"world": W,
           # what the transport was configured with (defaults unless set): the first record
           # from a real node says which RCCL and which knobs produced its numbers
           "env": {k: v for k, v in sorted(os.environ.items())
                   if k.startswith(("NCCL_", "RCCL_", "HSA_", "GPU_MAX_HW_QUEUES"))}}
    try:
        res["rccl_version"] = ".".join(str(x) for x in torch.cuda.nccl.version()) if on_gpu \
            else None
    except Exception:  # noqa: BLE001
        res["rccl_version"] = None

    def timed(fn):
        fn()
        if on_gpu:
            torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter()
        for _ in range(iters):
            fn()
        if on_gpu:
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / iters
        x = torch.tensor([dt], dtype=torch.float64, device=dev if on_gpu else "cpu")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return float(x.item())

    dt_bf = torch.bfloat16 if on_gpu else torch.float32
    esz = torch.empty((), dtype=dt_bf).element_size()

    def gather(mib):
        n = int(mib * 2**20 / esz) // W * W
        shard = torch.ones(n // W, dtype=dt_bf, device=dev)
        full = torch.empty(n, dtype=dt_bf, device=dev)
        t = timed(lambda: dist.all_gather_into_tensor(full, shard, group=gather_group))
        nbytes = n * esz
        return {"mib": round(nbytes / 2**20, 1), "ms": round(t * 1e3, 3),
                "algbw_gbps": round(nbytes / t / 1e9, 1),
                "busbw_gbps": round(nbytes / t / 1e9 * (W - 1) / W, 1)}

    def rscatter(numel):
        m = max(W, numel // W * W)
        g = torch.ones(m, dtype=torch.float32, device=dev)
        o = torch.empty(m // W, dtype=torch.float32, device=dev)
        t = timed(lambda: dist.reduce_scatter_tensor(o, g))
        return {"numel": m, "ms": round(t * 1e3, 3),
                "busbw_gbps": round(m * 4 / t / 1e9 * (W - 1) / W, 1)}

    if on_gpu:
        # which device pairs HIP reports peer access for (xGMI: every pair on an 8-GPU node);
        # the custom all-reduce's IPC mapping needs it (VERDICT r5 Next #7)
        try:
            n = torch.cuda.device_count()
            res["peer_access"] = {"devices": n, "matrix": [
                [1 if i == j else int(torch.cuda.can_device_access_peer(i, j)) for j in range(n)]
                for i in range(n)]}
        except Exception as e:  # noqa: BLE001
            res["peer_access"] = {"error": repr(e)[:200]}
    res["all_gather"] = dict(gather(unit_mb),
                             group="weight-gather" if gather_group is not None else "default")
    res["reduce_scatter"] = rscatter(bucket_numel)
    # size sweeps (bucket tuning data for the 7 xGMI links): the all-gather from a DeepSpeed
    # 5e7-element bucket (95 MiB bf16) down, the gradient reduce-scatter around the LoRA bucket
    scale = unit_mb / 386.0
    res["all_gather_sweep"] = [gather(mib * scale) for mib in (8, 32, 95)]
    res["reduce_scatter_sweep"] = [rscatter(int(n * scale)) for n in
                                   (500_000, 8_000_000, 16_777_216)]
    if on_gpu:
        try:
            from lumen.parallel.custom_ar import CustomAllReduce

            car = CustomAllReduce(None, dev, max_bytes=max(car_sizes))
            res["custom_ar_setup"] = {"ok": True, "world": car.world,
                                      "shared_device": bool(car.shared_device)}
            try:
                cal = car.calibrate(rccl_group=dist.group.WORLD, sizes=car_sizes, apply=False)
            finally:
                car.close()
            res["allreduce_us"] = cal["table"]
            res["allreduce_plan"] = cal["plan"]
        except Exception as e:  # noqa: BLE001 - the RCCL numbers stand
            res["allreduce_us"] = {"error": repr(e)[:300]}
            res.setdefault("custom_ar_setup", {"ok": False, "error": repr(e)[:300]})
    return res


def _max_unit(cfg) -> int:
    try:
        from lumen.parallel.memory_plan import llama_units

        return max(u["stored"] for u in llama_units(cfg))
    except Exception:  # noqa: BLE001 - non-Llama configs
        return 0


def _with_link_time(parts: dict, comm, world: int) -> dict:
    """Per partitioned schedule: the link time its per-step gather volume implies at the
    probe's measured all-gather bus bandwidth (each rank receives (W-1)/W of every gathered
    unit), next to the measured step and exposed wait -- comm-bound vs schedule-bound."""
    try:
        bus = comm["all_gather"]["busbw_gbps"] if comm else None
    except (KeyError, TypeError):
        bus = None
    out = {}
    for k, v in parts.items():
        v = dict(v)
        if bus and "gathered_mb_per_step" in v and world > 1:
            v["probe_busbw_gbps"] = bus
            v["implied_link_ms_per_step"] = round(
                v["gathered_mb_per_step"] * 1e6 * (world - 1) / world / (bus * 1e9) * 1e3, 2)
        out[k] = v
    return out


def _provenance():
    try:
        from lumen.ops._native import provenance

        return provenance()
    except Exception as e:  # noqa: BLE001
        return {"error": repr(e)[:200]}


def _claim_stdout():
    """The driver contract: stdout carries exactly one JSON line.  Keep a private handle on the
    real stdout for it and point fd 1 at stderr, so chatter from native libraries (gloo's
    connection messages, RCCL/HIP diagnostics) and from any Python print lands in stderr."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    json_out = _claim_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--micro_batch", type=int, default=8)
    ap.add_argument("--grad_accum", type=int, default=1)
    ap.add_argument("--seq_len", type=int, default=512)
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "ds_config_zero3_mi355x.json"))
    ap.add_argument("--lora_r", type=int, default=16)
    ap.add_argument("--dtype", default=None, choices=[None, "bf16", "fp16"],
                    help="override the config's precision (fp16: dynamic loss scaling)")
    ap.add_argument("--gradient_checkpointing", action="store_true")
    ap.add_argument("--profile_dir", default=None, help="write a torch.profiler trace here")
    ap.add_argument("--gemm_table", default=None,
                    help="TunableOp table to load ('off' = library heuristics); default "
                         "configs/tunableop/mi355x_gemms.csv when present")
    ap.add_argument("--tune_gemms", default=None, metavar="OUT_CSV",
                    help="tune the GEMM shapes during warmup and write the table at exit")
    ap.add_argument("--serve", dest="serve", action="store_true", default=True,
                    help="(default) at N=1 on a GPU, after the timed training steps: the serving "
                         "bench (Llama-2-7B TP=1, 256 requests x 512 in / 128 out) -> extra.serve")
    ap.add_argument("--no_serve", dest="serve", action="store_false")
    ap.add_argument("--serve_model", default=None, help="serving model (default: --model)")
    ap.add_argument("--partitioned", default="release,hybrid",
                    help="after the timed steps: 5 timed steps of each listed partitioned ZeRO-3 "
                         "schedule (release = the reference live budget 1e9 [configs/"
                         "ds_config_zero3.json]; hybrid = half the model resident) -> "
                         "extra.zero3_<schedule>; '' = none")
    ap.add_argument("--serve_tp", type=int, default=1,
                    help="at N > 1 on GPUs (1 = default): after the training sections, Llama-2-7B "
                         "served with TP = N (custom all-reduce over xGMI, 256 x 512 / 128, "
                         "engine mode) -> extra.serve_tp; 0 = skip; 2 = also on CPU / gloo "
                         "(tests)")
    ap.add_argument("--serve_tp_shape", default="256,512,128",
                    help="TP serving burst: requests,prompt_len,max_tokens")
    ap.add_argument("--serve_tp_deadline", type=float, default=420.0,
                    help="seconds the TP serving section may take: past it rank 0 prints the "
                         "JSON line with extra.serve_tp = an error, and every rank exits")
    ap.add_argument("--comm_probe", dest="comm_probe", action="store_true", default=True,
                    help="(default) at N > 1, after the timed steps: RCCL all-gather / "
                         "reduce-scatter bandwidth and custom vs RCCL all-reduce latency -> "
                         "extra.comm")
    ap.add_argument("--no_comm_probe", dest="comm_probe", action="store_false")
    ap.add_argument("--comm_probe_cpu_mb", type=float, default=8.0,
                    help="all-gather size of the probe on CPU / gloo runs (GPU: 386 MiB)")
    ap.add_argument("--partitioned_steps", type=int, default=5,
                    help="timed steps of each partitioned run (2 untimed warm-up steps first)")
    ap.add_argument("--wall_budget", type=float,
                    default=float(os.environ.get("LUMEN_BENCH_WALL_S", "520")),
                    help="seconds from process start for the whole run: an optional section "
                         "(comm probe, partitioned schedules, serving) whose estimate does not "
                         "fit in what is left is skipped and listed in extra.budget (the driver "
                         "kills the run at 600 s)")
    ap.add_argument("--box", dest="box", action="store_true", default=True,
                    help="(default, GPU) extra.box: clock / power sampled through the timed "
                         "region plus a fixed 8192^3 GEMM and a 4 GiB HBM read")
    ap.add_argument("--no_box", dest="box", action="store_false")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from lumen.ops._native import native, native_error

    if native() is None:
        from lumen.csrc.build import build

        build(verbose=False)
        import importlib

        import lumen.ops._native as nat

        nat._C, nat._err = None, None
        assert nat.native() is not None, nat.native_error()

    from lumen.lora import LoraConfig, apply_lora, count_parameters
    from lumen.models import build_model, get_config
    from lumen.parallel.dist import init
    from lumen.train.config import load_ds_config
    from lumen.train.engine import ZeroEngine

    # a hung collective must end the run (non-zero exit), not eat the driver's time budget
    os.environ.setdefault("LUMEN_DIST_TIMEOUT", "300")
    env = init()
    world = env.world_size
    from lumen.utils.gemm_tuning import load_tuned_gemms, start_gemm_tuning, tuned_entries

    if args.tune_gemms:
        start_gemm_tuning(args.tune_gemms)
        gemm_table = "tuning"
    else:
        gemm_table = "tuned" if load_tuned_gemms(args.gemm_table) else "heuristic"
    if world != args.gpus and env.is_main:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    ds = load_ds_config(args.config, args.micro_batch, args.grad_accum, world, 2e-4,
                        dtype_override=args.dtype)
    torch.manual_seed(1234)
    cfg = get_config(args.model)
    t_build = time.time()
    model = build_model(args.model, dtype=ds.torch_dtype, device=env.device, init="random", seed=0)
    apply_lora(model, LoraConfig(r=args.lora_r, lora_dropout=0.05))
    model.gradient_checkpointing = args.gradient_checkpointing
    model.train()
    n_tr, n_all = count_parameters(model)
    engine = ZeroEngine(model, ds, env)
    # overlapped reduce-scatter buckets of the LoRA gradients (16 MiB over xGMI at N > 1)
    dp_buckets = len(engine.flat.buckets)
    on_gpu = env.device.type == "cuda"
    if on_gpu:
        torch.cuda.synchronize()
    build_s = time.time() - t_build
    setup_s = time.time() - T_START  # process start -> engine ready (imports, init, build)
    coord = engine.coordinator
    # what RCCL itself sees: an all-reduce of ones over the default (gradient) group, and over
    # the ZeRO-3 weight-gather group when it is a separate communicator
    rccl_world = world
    gather_world = None
    if dist.is_initialized():
        one = torch.ones(1, device=env.device)
        dist.all_reduce(one)
        rccl_world = int(one.item())
        if engine.gather_group is not None:
            one = torch.ones(1, device=env.device)
            dist.all_reduce(one, group=engine.gather_group)
            gather_world = int(one.item())

    B, S = ds.micro_batch, args.seq_len
    n_batches = (args.warmup + args.steps) * ds.grad_accum
    g = torch.Generator(device="cpu").manual_seed(4321 + env.rank)
    batches = []
    for _ in range(min(n_batches, 8)):
        ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g)
        labels = torch.full_like(ids, -100)
        labels[:, :-1] = ids[:, 1:]
        batches.append({"input_ids": ids.to(env.device), "labels": labels.to(env.device),
                        "n_valid": int((labels != -100).sum())})

    # multi-rank: a hung collective ends the run with a diagnosis (exit 19) before the RCCL
    # watchdog's LUMEN_DIST_TIMEOUT, naming the LUMEN_ZERO3_SHARED_GROUP=1 escape hatch
    from lumen.utils.debug import StepWatchdog

    wd = (StepWatchdog.from_env(env.rank, coord, "training step")
          if world > 1 and not args.tune_gemms else None)

    def run_steps(n, offset):
        for s in range(n):
            for a in range(ds.grad_accum):
                b = batches[(offset + s * ds.grad_accum + a) % len(batches)]
                loss = engine.forward(b)
                engine.backward(loss)
                engine.step()
            if wd is not None:
                wd.kick()
        return loss

    def sync():
        from lumen.parallel.dist import barrier

        if on_gpu:
            torch.cuda.synchronize()
        if dist.is_initialized():
            barrier()  # device-bound barrier on RCCL, plain on gloo (CPU plumbing runs)
            if on_gpu:
                torch.cuda.synchronize()
        if wd is not None:
            wd.kick()

    loss = run_steps(args.warmup, 0)
    sync()
    if args.tune_gemms:  # timed steps use the tuned solutions, no tuning inside the timing
        import torch.cuda.tunable as tn

        tn.tuning_enable(False)
    prof = None
    if args.profile_dir and env.is_main:
        from torch.profiler import ProfilerActivity, profile

        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA])
        prof.__enter__()
    from lumen.bench.budget import WallBudget, partitioned_estimate_s
    from lumen.utils import boxcal

    def _agree_min(x: float) -> float:
        if not dist.is_initialized():
            return x
        t = torch.tensor([x], dtype=torch.float64 if not on_gpu else torch.float32,
                         device=env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return float(t.item())

    budget = WallBudget(args.wall_budget, T_START, _agree_min)
    # heartbeat on stderr once a minute (which section, how long): a long section over a slow
    # transport (a shared-GPU rehearsal's loopback RCCL) reads as progress, not as a hang
    import threading as _th

    def _heartbeat():
        while True:
            time.sleep(60)
            o = budget._open
            print(f"[bench] rank {env.rank}: {time.time() - T_START:.0f} s, section "
                  f"{o['section'] if o else 'headline / between sections'}", file=sys.stderr,
                  flush=True)

    _th.Thread(target=_heartbeat, daemon=True, name="bench-heartbeat").start()
    hwmon = boxcal.gpu_hwmon(env.device) if (on_gpu and args.box) else None
    sampler = boxcal.HwmonSampler(hwmon).start() if (on_gpu and args.box) else None
    # every timed step must really update the adapters: a non-finite gradient makes the fused
    # AdamW skip the step on the device (a NaN-producing kernel would otherwise time as "fast")
    sk0 = engine.skipped_steps
    gb0 = coord.gathered_bytes if coord else 0
    if coord is not None:
        coord.pop_exposed_wait_ms()
        coord.track_waits = True  # timing events around every gather wait (exposed comm)
    t1 = time.perf_counter()
    loss = run_steps(args.steps, args.warmup)
    sync()
    dt = time.perf_counter() - t1
    timed_box = sampler.stop() if sampler is not None else None
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(args.profile_dir, "bench_trace.json"))
        with open(os.path.join(args.profile_dir, "bench_ops.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    exposed_ms = coord.pop_exposed_wait_ms() if coord is not None else 0.0
    peak_gb = torch.cuda.max_memory_allocated() / 1e9 if on_gpu else 0.0
    # max over ranks of: timed region, exposed gather wait, peak HBM
    t = torch.tensor([dt, exposed_ms, peak_gb], dtype=torch.float64 if not on_gpu
                     else torch.float32, device=env.device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, exposed_ms, peak_gb = (float(x) for x in t.tolist())
    final_loss = float(loss.item())
    skipped = engine.skipped_steps - sk0
    if skipped and env.is_main:
        print(f"[bench] WARNING: {skipped} of {args.steps} timed optimizer steps were skipped "
              "(non-finite gradients): this number is not a valid training throughput",
              file=sys.stderr)
    tokens = world * B * ds.grad_accum * S * args.steps
    value = tokens / dt
    if coord is None:
        par = f"dp{world}-zero{ds.stage}"
    elif coord.identity:
        par = f"dp{world}-zero{ds.stage}(world-1 partition = whole model: no gathers)"
    elif coord.keep:
        # frozen base weights gathered once, then resident (replicated): per-step traffic is
        # the LoRA gradient reduce-scatter + adapter publish; the partitioned schedules are
        # timed separately (extra.zero3_release / extra.zero3_hybrid)
        par = f"dp{world}-zero{ds.stage}-keep(frozen weights gathered once, resident)"
    else:
        par = f"dp{world}-zero{ds.stage}-{coord.schedule}"
    gathered_mb = ((coord.gathered_bytes - gb0) / 1e6 / args.steps) if coord else 0.0
    gathered_total_mb = coord.gathered_bytes / 1e6 if coord else 0.0
    zstats = coord.stats() if coord else None
    if wd is not None:
        wd.close()
    box = None
    if on_gpu and args.box:
        # fixed work on this box, same process and lease, right after the timed region: a slow
        # record is a slow box when these ran slow too (max over ranks at N > 1)
        try:
            fixed = boxcal.fixed_work(env.device, hwmon=hwmon)
            if dist.is_initialized():
                v = torch.tensor([fixed["gemm"]["ms_med"],
                                  fixed.get("hbm_read", {}).get("ms_med", 0.0)],
                                 dtype=torch.float32, device=env.device)
                dist.all_reduce(v, op=dist.ReduceOp.MAX)
                fixed["max_over_ranks"] = {"gemm_ms_med": round(float(v[0]), 3),
                                           "hbm_read_ms_med": round(float(v[1]), 3)}
            box = boxcal.box_record(env.device, timed_box, fixed)
        except Exception as e:  # noqa: BLE001 - keep the headline result
            box = {"error": repr(e)[:300], "timed_region": timed_box}
    ms_step = dt / args.steps * 1000
    comm = None
    if world > 1 and args.comm_probe and budget.allow("comm_probe", 30.0 if on_gpu else 10.0):
        # after (and outside) the timed region: the transport's own numbers
        try:
            comm = run_comm_probe(env, engine.gather_group,
                                  unit_mb=386.0 if on_gpu else args.comm_probe_cpu_mb)
        except Exception as e:  # noqa: BLE001 - keep the headline result
            comm = {"error": repr(e)[:300]}
            raise  # ranks may disagree on where they failed: do not continue collectives
        budget.done("comm_probe")
    serve = serve_engine = serve_chunked = serve_sampled = None
    parts = {}
    want_parts = [x for x in args.partitioned.split(",") if x] if ds.stage == 3 else []
    if want_parts or (args.serve and world == 1 and on_gpu):
        engine.close()
        del engine, model, coord
        engine = None
        import gc

        gc.collect()
        if on_gpu:
            torch.cuda.empty_cache()
    for sched in want_parts:
        # the partitioned ZeRO-3 paths, timed after (and outside) the headline region
        # hybrid = release's ring budget PLUS resident units: at least the reference live budget
        # and one decoder unit beyond it (half the model on Llama-2-7B), so a shallow model
        # never runs a hybrid whose ring is smaller than release's (r4 world-8 rehearsal:
        # 2,147 vs 1,338 MB gathered per step at half of a 2-layer model)
        ml = 1e9 if sched == "release" else max(0.5 * cfg.num_params(), 1e9 + _max_unit(cfg))
        est = partitioned_estimate_s(ms_step, args.partitioned_steps,
                                     min(2, args.partitioned_steps), build_s)
        if not budget.allow(f"zero3_{sched}", est):
            parts[sched] = {"skipped": "wall budget", "est_s": round(est, 1)}
            continue
        try:
            parts[sched] = run_partitioned(args, env, ds, batches, sched, ml,
                                           steps=args.partitioned_steps,
                                           warmup=min(2, args.partitioned_steps))
        except Exception as e:  # noqa: BLE001 - keep the headline result
            parts[sched] = {"error": repr(e)[:300]}
            if world > 1:
                raise  # ranks may disagree on where they failed: do not continue collectives
        budget.done(f"zero3_{sched}")
    if args.serve and world == 1 and on_gpu:
        # second half of the BASELINE metric ("serve tok/s + p50 TTFT"), after the timed
        # training region: the training model and engine are freed first
        del batches
        if budget.allow("serve", 60.0):
            serve, serve_engine, serve_chunked, serve_sampled = run_serve_bench(args)
            budget.done("serve")
        else:
            serve = {"skipped": "wall budget"}
    out = None
    if env.is_main:
        from lumen.train.trainer import model_flops_per_token

        tflops = value / world * model_flops_per_token(cfg, S) / 1e12
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_TOK_S, 2),
            "dtype": ds.dtype,
            "data": f"synthetic (uniform random token ids, seq {S}); random-init weights",
            "config": {
                "model": cfg.name,
                "global_batch": B * ds.grad_accum * world,
                "micro_batch": B,
                "grad_accum": ds.grad_accum,
                "seq_len": S,
                "parallelism": par,
                "lora": f"r={args.lora_r} alpha={2 * args.lora_r} dropout=0.05 q,k,v,o",
                "trainable_params": n_tr,
                "total_params": n_all,
            },
            "extra": {
                "tflops_per_gpu": round(tflops, 1),
                "samples_per_second": round(B * ds.grad_accum * world * args.steps / dt, 2),
                "peak_hbm_gb_max_rank": round(peak_gb, 2),
                "final_loss": round(final_loss, 4),
                "timed_steps_skipped_nonfinite": skipped,
                "setup_s": round(setup_s, 2),
                "model_build_s": round(build_s, 3),
                "rccl_world": rccl_world,
                "gather_group_world": gather_world,
                "backend": env.backend,
                "zero3": zstats,
                "dp_grad_buckets": dp_buckets,
                # keep schedule: the frozen weights are gathered once (warm-up), 0 per timed step
                "zero3_gathered_mb_total": round(gathered_total_mb, 1),
                "zero3_gathered_mb_per_step": round(gathered_mb, 1),
                "zero3_received_mb_per_step_per_rank": round(gathered_mb * (world - 1) / world, 1),
                "zero3_exposed_wait_ms_per_step_max_rank": round(exposed_ms / args.steps, 2),
                "baseline_tok_s": BASELINE_TOK_S,
                "gemm_algos": gemm_table,
                "native_build": _provenance(),
                "gemm_table_entries": tuned_entries() if gemm_table != "heuristic" else 0,
                "comm": comm,
                **{f"zero3_{k}": v for k, v in _with_link_time(parts, comm, world).items()},
                "serve": serve,
                "serve_engine": serve_engine,
                "serve_chunked": serve_chunked,
                "serve_sampled": serve_sampled,
                "box": box,
            },
        }
    import threading

    timer = None
    printed = [False]
    print_lock = threading.Lock()

    def _print_once():
        with print_lock:
            if out is not None and not printed[0]:
                print(json.dumps(out), file=json_out, flush=True)
                printed[0] = True

    tp_deadline = args.serve_tp_deadline
    run_tp = bool(args.serve_tp and world > 1 and (on_gpu or args.serve_tp == 2))
    if run_tp:
        # the TP section's own deadline is cut to what the wall budget leaves (minus the
        # closing barrier and teardown); below a minute it is not started at all
        tp_deadline = min(args.serve_tp_deadline, budget.left() - 20.0)
        min_tp = 60.0 if on_gpu else 1.0
        if tp_deadline < min_tp and args.serve_tp_deadline >= min_tp:
            budget.skipped.append({"section": "serve_tp", "est_s": min_tp,
                                   "left_s": round(tp_deadline + 20.0, 1)})
            run_tp = False
            if out is not None:
                out["extra"]["serve_tp"] = {"skipped": "wall budget"}
        else:
            tp_deadline = max(tp_deadline, min(args.serve_tp_deadline, 0.01))
    if out is not None:
        out["extra"]["budget"] = budget.record()
        if run_tp:
            out["extra"]["budget"]["serve_tp_deadline_s"] = round(tp_deadline, 1)
    if run_tp:
        # TP = N serving over the N GPUs.  A hung collective must not cost the training record:
        # past the deadline (TP section + closing barrier) rank 0 prints the JSON line with the
        # error (unless it already did) and every rank exits
        if engine is not None:
            engine.close()
            engine = None

        def _deadline():
            if out is not None and not printed[0]:
                out["extra"]["serve_tp"] = {"error": f"timed out after {tp_deadline:.1f} s"}
            _print_once()
            os._exit(0)

        timer = threading.Timer(tp_deadline + (0 if env.is_main else 15), _deadline)
        timer.daemon = True
        timer.start()
        try:
            stp = run_serve_tp(args, env)
        except Exception as e:  # noqa: BLE001 - keep the training record
            stp = {"error": repr(e)[:500]}
        if out is not None:
            out["extra"]["serve_tp"] = stp
    _print_once()
    if engine is not None:
        engine.close()  # drain in-flight (next-step) gathers before teardown
    if dist.is_initialized():
        from lumen.parallel.dist import barrier

        try:
            barrier()
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            if timer is not None:
                # a peer gave up on the TP section (its deadline); rank 0's record is out
                os._exit(0)
            raise
    if timer is not None:
        timer.cancel()


if __name__ == "__main__":
    main()
