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

    env = init(device="cpu")
    raw = {"zero_optimization": {"stage": stage, "reduce_bucket_size": 3000,
                                 "stage3_param_persistence_threshold": 100,
                                 "stage3_max_live_parameters": (extra or {}).get("max_live", 1e9)},
           "bf16": {"enabled": False}}
    if extra and extra.get("offload"):
        raw["zero_optimization"]["offload_optimizer"] = {"device": "cpu", "pin_memory": False}
    ds = load_ds_config(raw, micro, accum, world, 1e-2, dtype_override="fp32")
    a = TrainArgs(model_name=model, synthetic=True, synthetic_samples=64, max_length=16,
                  per_device_train_batch_size=micro, gradient_accumulation_steps=accum,
                  max_steps=steps, logging_steps=1, lora_r=4, lora_dropout=0.0,
                  save_strategy="no", save_final=False, output_dir=os.path.join(outdir, "ck"),
                  seed=7)
    t = Trainer(a, ds, env, printer=lambda *x, **k: None)
    res = t.train()
    if rank == 0:
        sd = adapter_state_dict(t.model)
        torch.save({"sd": sd, "losses": [r["loss"] for r in t.log_history], "res": res},
                   os.path.join(outdir, f"result_stage{stage}_w{world}.pt"))
    shutdown()


def serve_tp_worker(rank, world, port, outdir, loras=None):
    """TP serving on gloo: rank 0 runs the engine, rank 1 the worker loop; greedy outputs of
    rank 0 are saved for comparison with a single-process engine."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import torch

    torch.set_num_threads(1)
    from lumen.parallel.dist import init, shutdown
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams
    from lumen.serve.tp import worker_loop

    init(device="cpu")
    model = _tp_test_model()
    cfg = EngineConfig(model="tiny-llama-gqa", device="cpu", max_model_len=128, block_size=4,
                       use_graphs=False, num_blocks=128, tp_size=world, lora_modules=loras)
    eng = LLMEngine(cfg, model=model)
    if rank == 0:
        prompts = [[5, 9, 33, 7], list(range(3, 30)), [42, 43]]
        sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
        names = list(loras or {}) + [None] * 3
        seqs = [eng.add_request(p, SamplingParams(**vars(sp)), lora=names[i])
                for i, p in enumerate(prompts)]
        while any(not s.finished for s in seqs):
            eng.step()
        eng.shutdown()
        torch.save([s.output_ids for s in seqs], os.path.join(outdir, "tp_out.pt"))
    else:
        worker_loop(eng.runner)
    shutdown()


def _tp_test_model():
    import torch

    from lumen.models import build_model

    m = build_model("tiny-llama-gqa", dtype=torch.float32, device="cpu", init="random", seed=1)
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
