"""Steady-state 256-row decode step of Llama-2-7B serving (TP=1, graph replay): time per step
after a prefill-first burst, and -- under rocprofv3 --kernel-trace -- a kernel table of the
decode steps alone (they follow a 0.5 s idle gap the post-processor looks for:
scripts/tools/decode_table.py).

    python scripts/probes/decode_step_probe.py [--kv fp8] [--steps 48] [--rows 256]"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--kv", default="auto")
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--prompt", type=int, default=576)
    ap.add_argument("--steps", type=int, default=48)
    a = ap.parse_args()
    import torch

    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model=a.model, dtype="bf16", max_model_len=1024,
                                 max_num_seqs=a.rows, max_num_batched_tokens=16384,
                                 scheduling_policy="prefill_first", init="random",
                                 kv_cache_dtype=a.kv))
    rng = random.Random(0)
    V = eng.model_config.vocab_size
    seqs = [eng.add_request([rng.randrange(3, V) for _ in range(a.prompt)],
                            SamplingParams(max_tokens=a.steps + 40, temperature=0.0,
                                           ignore_eos=True)) for _ in range(a.rows)]
    while any(len(s.output_ids) < 1 for s in seqs):      # prefill (and first decode steps)
        eng.step()
    for _ in range(8):                                     # graph capture / warm decode
        eng.step()
    torch.cuda.synchronize()
    time.sleep(0.5)                                        # the gap the trace splitter finds
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    ctx = sum(s.length for s in seqs) / len(seqs)
    kv_bytes = 2 * eng.model_config.num_hidden_layers * eng.model_config.hidden_size * (
        1 if a.kv == "fp8" else 2) * ctx * a.rows
    print(json.dumps({"ms_per_decode_step": round(dt * 1e3, 3), "rows": a.rows,
                      "mean_context_end": round(ctx, 1), "kv": a.kv,
                      "kv_gb_per_step": round(kv_bytes / 1e9, 2)}))
    eng.shutdown()


if __name__ == "__main__":
    main()
