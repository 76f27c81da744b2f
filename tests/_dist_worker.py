"""Worker for multi-process CPU/gloo tests (importable so torch.multiprocessing can spawn it)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def train_worker(rank, world, port, stage, outdir, model="tiny-llama", micro=2, accum=1,
                 steps=3, extra=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import torch

    torch.set_num_threads(1)
    from lumen.lora import adapter_state_dict
    from lumen.parallel.dist import init, shutdown
    from lumen.train.config import load_ds_config
    from lumen.train.trainer import TrainArgs, Trainer

    saved_env = {k: os.environ.get(k) for k in ("LUMEN_ZERO3_SCHEDULE", "LUMEN_ZERO3_SINGLE")}
    saved_env.update({k: os.environ.get(k) for k in (extra or {}).get("env", {})})
    os.environ.update((extra or {}).get("env", {}))
    if extra and extra.get("schedule"):
        os.environ["LUMEN_ZERO3_SCHEDULE"] = extra["schedule"]
    if extra and extra.get("single"):
        os.environ["LUMEN_ZERO3_SINGLE"] = "1"
    if (extra or {}).get("device") == "cuda" and world > 1:
        os.environ["LUMEN_SHARED_GPU_REHEARSAL"] = "1"  # RCCL ranks share the one GPU
        os.environ.setdefault("LUMEN_DIST_TIMEOUT", "120")  # a hung collective fails the test
    env = init(device=(extra or {}).get("device", "cpu"))
    raw = {"zero_optimization": {"stage": stage, "reduce_bucket_size": 3000,
                                 "stage3_param_persistence_threshold": 100,
                                 "stage3_max_live_parameters": (extra or {}).get("max_live", 1e9)},
           "bf16": {"enabled": False}}
    if extra and extra.get("offload"):
        raw["zero_optimization"]["offload_optimizer"] = {"device": "cpu", "pin_memory": False}
    if extra and extra.get("offload_param"):
        raw["zero_optimization"]["offload_param"] = {"device": "cpu", "pin_memory": False}
    if extra and extra.get("prefetch") is not None:
        raw["zero_optimization"]["stage3_prefetch_bucket_size"] = extra["prefetch"]
    if extra and extra.get("reuse") is not None:
        raw["zero_optimization"]["stage3_max_reuse_distance"] = extra["reuse"]
    ds = load_ds_config(raw, micro, accum, world, 1e-2,
                        dtype_override=(extra or {}).get("dtype", "fp32"))
    ex = extra or {}
    a = TrainArgs(model_name=model, synthetic=True, synthetic_samples=64, max_length=16,
                  per_device_train_batch_size=micro, gradient_accumulation_steps=accum,
                  max_steps=steps, logging_steps=1, lora_r=4, lora_dropout=0.0,
                  save_strategy="steps" if ex.get("save_steps") else "no",
                  save_steps=ex.get("save_steps", 100), resume_from_checkpoint=ex.get(
                      "resume", False), save_final=False,
                  output_dir=ex.get("ckdir") or os.path.join(outdir, "ck"),
                  seed=7, gradient_checkpointing=(extra or {}).get("gc", False),
                  fuse_accumulation=ex.get("fuse", True), synthetic_min_len=ex.get("min_len"))
    try:
        t = Trainer(a, ds, env, printer=lambda *x, **k: None)
        res = t.train()
        if extra and extra.get("single"):
            assert t.engine.coordinator is not None
    finally:
        for k, v in saved_env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if rank == 0:
        sd = adapter_state_dict(t.model)
        co = t.engine.coordinator
        stats = dict(co.stats(), gathers=co.gathers) if co is not None else None
        if stats is not None:
            stats["gather_group_separate"] = t.engine.gather_group is not None
        torch.save({"sd": sd, "losses": [r["loss"] for r in t.log_history], "res": res,
                    "zero3": stats, "fusion": dict(t.fusion_stats),
                    "async_offload": t.engine.async_off is not None},
                   os.path.join(outdir, f"result_stage{stage}_w{world}.pt"))
    shutdown()


def serve_tp_worker(rank, world, port, outdir, loras=None, async_sched=True, cap=None,
                    extra=None):
    """TP serving on gloo: rank 0 runs the engine, rank 1 the worker loop; greedy outputs of
    rank 0 are saved for comparison with a single-process engine."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import torch

    torch.set_num_threads(1)
    from lumen.parallel.dist import init, shutdown
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams
    import lumen.serve.tp as tp_mod
    from lumen.serve.tp import worker_loop

    if cap is not None:  # small inline host capacity: prefill steps take the two-message path
        tp_mod.HOST_CAP = cap

    init(device="cpu")
    model = _tp_test_model()
    cfg = EngineConfig(model="tiny-llama-gqa", device="cpu", max_model_len=128, block_size=4,
                       use_graphs=False, num_blocks=128, tp_size=world, lora_modules=loras,
                       async_scheduling=async_sched, **(extra or {}))
    eng = LLMEngine(cfg, model=model)
    if rank == 0:
        prompts = [[5, 9, 33, 7], list(range(3, 30)), [42, 43]]
        if (extra or {}).get("enable_prefix_caching"):
            # a finished request's blocks: the later prompts share its first 24 tokens
            warm = eng.add_request(list(range(3, 30)) + [1], SamplingParams(
                max_tokens=2, temperature=0.0, ignore_eos=True))
            while not warm.finished:
                eng.step()
        sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
        names = list(loras or {}) + [None] * 3
        seqs = [eng.add_request(p, SamplingParams(**vars(sp)), lora=names[i])
                for i, p in enumerate(prompts)]
        while any(not s.finished for s in seqs):
            eng.step()
        eng.shutdown()
        assert eng.async_sched == (async_sched and not (extra or {}).get("num_speculative_tokens"))
        if (extra or {}).get("enable_prefix_caching"):
            assert eng.blocks.hit_tokens > 0
        torch.save([s.output_ids for s in seqs], os.path.join(outdir, "tp_out.pt"))
    else:
        worker_loop(eng.runner)
    shutdown()


def _tp_test_model(name="tiny-llama-gqa"):
    import torch

    from lumen.models import build_model

    m = build_model(name, dtype=torch.float32, device="cpu", init="random", seed=1)
    with torch.no_grad():
        for p in m.parameters():
            if p.dim() == 2:
                p.mul_(5.0)
    m.eval()
    return m


def eval_worker(rank, world, port, outdir):
    """Data-parallel evaluate_loss on a fixed tiny model; rank 0 writes the result."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import json

    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    from lumen.data.collator import CausalLMCollator
    from lumen.data.datasets import SyntheticTokenDataset
    from lumen.eval import evaluate_loss
    from lumen.models import build_model

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    m = build_model("tiny-llama", dtype=torch.float32, device=torch.device("cpu"), seed=3)
    ds = SyntheticTokenDataset(7, 24, m.config.vocab_size, seed=5, min_len=8)
    res = evaluate_loss(m, ds, CausalLMCollator(pad_id=2), batch_size=2, rank=rank, world=world)
    if rank == 0:
        with open(os.path.join(outdir, f"eval_w{world}.json"), "w") as f:
            json.dump(res, f)
    if world > 1:
        dist.destroy_process_group()


def car_worker(rank, world, port, outdir):
    """Custom all-reduce on ONE GPU shared by `world` processes (gloo only exchanges the IPC
    handles): every dtype / size / one-shot / two-shot / graph case checked bit-exactly against
    the same f32 sum in rank order, computed on the host."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import json
    import time

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lumen.parallel.custom_ar import CustomAllReduce

    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, dev, max_bytes=4 << 20, timeout_s=20.0)
    res = {"cases": [], "timing_us": {}}

    def inputs(case, n, dt):
        xs = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * case + q)).to(dt)
              for q in range(world)]
        acc = xs[0].float()
        for q in range(1, world):
            acc = acc + xs[q].float()
        return xs[rank], acc.to(dt)

    case = 0
    for dt, n in ((torch.bfloat16, 8), (torch.bfloat16, 4096), (torch.float32, 12345 * 8),
                  (torch.float16, 65536), (torch.bfloat16, 1 << 20), (torch.float32, 8 * 1001)):
        for two in (False, True):
            for blocks in (None, 1, 7):
                case += 1
                x, want = inputs(case, n, dt)
                xd = x.to(dev)
                inplace = case % 2 == 0
                out = xd if inplace else torch.empty_like(xd)
                car.all_reduce(xd, out=out, two_shot=two, blocks=blocks)
                got = out.cpu()
                bad = int((got.float() != want.float()).sum())
                res["cases"].append({"dtype": str(dt), "n": n, "two_shot": two, "blocks": blocks,
                                     "inplace": inplace, "mismatches": bad})
    # hipGraph capture + replay with new inputs each time
    n = 65536
    xs = torch.empty(n, dtype=torch.bfloat16, device=dev)
    ys = torch.empty_like(xs)
    xs.fill_(1.0)
    car.all_reduce(xs, out=ys)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            car.all_reduce(xs, out=ys)
    graph_bad = 0
    for it in range(3):
        case += 1
        x, want = inputs(case, n, torch.bfloat16)
        xs.copy_(x.to(dev))
        g.replay()
        graph_bad += int((ys.cpu().float() != want.float()).sum())
    res["graph_mismatches"] = graph_bad
    # latency on a shared GPU (not an xGMI number: both ranks sit on one device)
    for nbytes in (8 << 10, 256 << 10, 2 << 20):
        t = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=dev)
        for _ in range(5):
            car.all_reduce(t)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            car.all_reduce(t)
        torch.cuda.synchronize()
        res["timing_us"][str(nbytes)] = (time.perf_counter() - t0) / 50 * 1e6
    car.check()
    res["err"] = 0
    dist.barrier()
    car.close()
    if rank == 0:
        with open(os.path.join(outdir, "car.json"), "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


def serve_tp_gpu_worker(rank, world, port, outdir, backend="gloo", model_name="tiny-llama-gqa"):
    """TP=world serving with every rank on the ONE GPU (``backend`` carries the step payload and
    the vocab gather -- gloo, or RCCL under LUMEN_SHARED_GPU_REHEARSAL; the row-parallel sums
    take the custom IPC all-reduce, so decode buckets run as hipGraphs).  Rank 0 saves greedy
    outputs + which paths were active.  world 1: the TP=1 reference run."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE="1")
    if backend == "nccl" and world > 1:
        os.environ["LUMEN_SHARED_GPU_REHEARSAL"] = "1"
        os.environ.setdefault("LUMEN_DIST_TIMEOUT", "120")
    import torch

    from lumen.parallel.dist import init, shutdown
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams
    from lumen.serve.tp import worker_loop

    init(backend=backend, device="cuda")
    model = _tp_test_model(model_name).to("cuda")
    model = model.to(torch.bfloat16)  # the paged-KV kernels are 16-bit
    cfg = EngineConfig(model=model_name, device="cuda:0", dtype="bf16", max_model_len=128,
                       block_size=16, use_graphs=True, num_blocks=64, tp_size=world,
                       max_num_seqs=8)
    eng = LLMEngine(cfg, model=model)
    info = {"car": eng.runner.car is not None, "graphs": eng.runner.use_graphs}
    if rank == 0:
        prompts = [[5, 9, 33, 7], list(range(3, 30)), [42, 43]]
        sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
        seqs = [eng.add_request(p, SamplingParams(**vars(sp))) for p in prompts]
        while any(not s.finished for s in seqs):
            eng.step()
        eng.shutdown()
        info["captured"] = sorted(eng.runner._graphs)
        info["car_calls"] = eng.runner.car.calls if eng.runner.car is not None else 0
        if eng.runner.car is not None:
            eng.runner.car.check()
        info["backend"] = (torch.distributed.get_backend()
                           if torch.distributed.is_initialized() else "none")
        torch.save({"out": [s.output_ids for s in seqs], "info": info},
                   os.path.join(outdir, "tp_gpu_out.pt"))
    else:
        worker_loop(eng.runner)
    if eng.runner.car is not None:
        # every rank's barrier record: the longest wait for a peer (> 1 ms) and, after a
        # timeout, which barrier waited for which rank (tests/test_rccl_gpu.py reports them)
        import json

        with open(os.path.join(outdir, f"car_diag_{rank}.json"), "w") as f:
            json.dump(eng.runner.car.diagnostics(), f)
    shutdown()


def car_skew_worker(rank, world, port, outdir, delay_s, timeout_s):
    """Custom all-reduce with rank ``world - 1`` arriving ``delay_s`` late on the host (the
    others' kernels already spinning in the first barrier): within the deadline the sum is exact
    and the early ranks record the wait; past it the early ranks raise CollectiveTimeout naming
    the late rank and the barrier, while the late rank still computes the right sum."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import json
    import time

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lumen.parallel.custom_ar import CollectiveTimeout, CustomAllReduce

    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, dev, max_bytes=1 << 20, timeout_s=timeout_s)
    x = torch.full((4096,), float(rank + 1), dtype=torch.bfloat16, device=dev)
    torch.cuda.synchronize()
    dist.barrier()
    if rank == world - 1:
        time.sleep(delay_s)
    t0 = time.perf_counter()
    car.all_reduce(x)
    torch.cuda.synchronize()
    res = {"rank": rank, "wall_s": time.perf_counter() - t0,
           "exact": bool((x.float() == world * (world + 1) / 2).all())}
    try:
        car.poll()
        res["timeout"] = None
    except CollectiveTimeout as e:
        res["timeout"] = str(e)
    res["diag"] = car.diagnostics()
    with open(os.path.join(outdir, f"skew_{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    car.close()
    dist.destroy_process_group()


def car_gather_worker(rank, world, port, outdir):
    """Custom column all-gather ([R, Vs] shards -> [R, W*Vs]) on one shared GPU, incl. graph."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import json

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lumen.parallel.custom_ar import CustomAllReduce

    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, dev, max_bytes=2 << 20, timeout_s=20.0)
    bad = 0
    for i, (R, Vs, dt, blocks) in enumerate(((1, 8, torch.bfloat16, None), (3, 256, torch.float32, 5),
                                             (37, 4000, torch.bfloat16, None),
                                             (256, 2000, torch.float16, 128))):
        shards = [torch.randn(R, Vs, generator=torch.Generator().manual_seed(100 * i + q)).to(dt)
                  for q in range(world)]
        want = torch.cat(shards, 1)
        got = car.all_gather_cols(shards[rank].to(dev), blocks=blocks).cpu()
        bad += int((got != want).sum())
    x = torch.zeros(16, 512, dtype=torch.bfloat16, device=dev)
    car.all_gather_cols(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(torch.cuda.Stream()):
        with torch.cuda.graph(g):
            y = car.all_gather_cols(x)
    for it in range(2):
        shards = [torch.full((16, 512), float(10 * it + q), dtype=torch.bfloat16)
                  for q in range(world)]
        x.copy_(shards[rank].to(dev))
        g.replay()
        bad += int((y.cpu() != torch.cat(shards, 1)).sum())
    car.check()
    dist.barrier()
    car.close()
    if rank == 0:
        with open(os.path.join(outdir, "gather.json"), "w") as f:
            json.dump({"mismatches": bad}, f)
    dist.destroy_process_group()


def car_timeout_worker(rank, world, port, outdir):
    """Rank 1 skips a custom all-reduce: rank 0's barrier must give up after its deadline, set
    the pinned host error word, and ``poll()`` must raise (no silent half-reduced result)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import json

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lumen.parallel.custom_ar import CollectiveTimeout, CustomAllReduce

    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, dev, max_bytes=1 << 20, timeout_s=2.0)
    x = torch.ones(4096, dtype=torch.bfloat16, device=dev)
    car.all_reduce(x)          # a good call first: both ranks take part
    torch.cuda.synchronize()
    car.poll()
    res = {"first": float(x[0])}
    dist.barrier()
    if rank == 0:
        car.all_reduce(x)      # rank 1 never joins this one
        torch.cuda.synchronize()
        try:
            car.poll()
            res["raised"] = False
        except CollectiveTimeout:
            res["raised"] = True
        res["err_word"] = int(car.C.car_err(car._sig))
    dist.barrier()
    car.close()
    if rank == 0:
        with open(os.path.join(outdir, "car_timeout.json"), "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


def rccl_probe_worker(rank, world, port, outdir):
    """scripts/probes/rccl_probe.py as a spawned rank: RCCL collectives with every rank on the
    box's one GPU (LUMEN_SHARED_GPU_REHEARSAL)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world),
                      LUMEN_SHARED_GPU_REHEARSAL="1", LUMEN_DIST_TIMEOUT="120")
    sys.path.insert(0, os.path.join(ROOT, "scripts", "probes"))
    import rccl_probe

    rccl_probe.main()
    with open(os.path.join(outdir, f"probe_ok_{rank}"), "w") as f:
        f.write("ok")


def car_calibrate_worker(rank, world, port, outdir, delay_s, timeout_s):
    """``CustomAllReduce.calibrate`` on every rank; with ``delay_s`` > 0 the last rank starts it
    late, so an early rank's first barrier times out: every rank must then raise (collectively,
    after the shared max-reduction) instead of one raising and its peers hanging."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    import json
    import time

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lumen.parallel.custom_ar import CollectiveTimeout, CustomAllReduce

    dev = torch.device("cuda", 0)
    car = CustomAllReduce(dist.group.WORLD, dev, max_bytes=1 << 20, timeout_s=timeout_s)
    dist.barrier()
    if rank == world - 1 and delay_s > 0:
        time.sleep(delay_s)
    res = {"rank": rank}
    t0 = time.perf_counter()
    try:
        cal = car.calibrate(rccl_group=None, sizes=(8 << 10, 256 << 10), iters=3, warmup=1,
                            apply=False)
        res["table"], res["plan"], res["error"] = cal["table"], cal["plan"], None
    except CollectiveTimeout as e:
        res["error"] = str(e)
    res["wall_s"] = time.perf_counter() - t0
    with open(os.path.join(outdir, f"cal_{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    car.close()
    dist.destroy_process_group()


def car_fallback_worker(rank, world, port, outdir, delay_s, timeout_s):
    """``maybe_custom_allreduce`` when its calibration times out (the last rank starts late):
    every rank must get None back (RCCL serves the TP reductions) instead of an exception that
    aborts engine startup."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", LUMEN_CAR_CALIBRATE="always",
                      LUMEN_CAR_TIMEOUT=str(timeout_s))
    import json
    import time

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import lumen.parallel.custom_ar as car_mod

    orig = car_mod.CustomAllReduce.calibrate

    def late_calibrate(self, *a, **k):
        if rank == world - 1 and delay_s > 0:
            time.sleep(delay_s)
        return orig(self, *a, **k)

    car_mod.CustomAllReduce.calibrate = late_calibrate
    res = {"rank": rank}
    try:
        car = car_mod.maybe_custom_allreduce(dist.group.WORLD, torch.device("cuda", 0), 1 << 20)
        res["car"] = car is not None
        res["error"] = None
        if car is not None:
            car.close()
    except Exception as e:  # noqa: BLE001
        res["error"] = repr(e)
    with open(os.path.join(outdir, f"fb_{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()
