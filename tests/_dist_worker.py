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
