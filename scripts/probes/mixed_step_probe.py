"""Steady-state mixed (chunked-prefill) step of Llama-2-7B serving: ``--decode`` sequences decode
while new 512-token prompts keep arriving, so every step under the chunked policy carries
``--decode`` decode rows plus (budget - decode) prefill tokens -- the step the
``extra.serve_chunked`` burst spends half its time in (profiles/r4_serve_policy: 68 mixed steps
of ~1900 prefill tokens + ~130 decode rows).  Prints ms per step; under rocprofv3 --kernel-trace
the timed steps follow a 0.5 s idle gap (scripts/tools/gap_table.py).

    python scripts/probes/mixed_step_probe.py [--decode 132] [--budget 2048] [--steps 24]"""
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
    ap.add_argument("--decode", type=int, default=132)
    ap.add_argument("--budget", type=int, default=2048)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--graphs", type=int, default=1)
    a = ap.parse_args()
    import torch

    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model=a.model, dtype="bf16", max_model_len=1024,
                                 max_num_seqs=512, max_num_batched_tokens=a.budget,
                                 scheduling_policy="chunked", init="random",
                                 use_graphs=bool(a.graphs)))
    rng = random.Random(0)
    V = eng.model_config.vocab_size

    def add(n, max_tokens):
        return [eng.add_request([rng.randrange(3, V) for _ in range(a.prompt)],
                                SamplingParams(max_tokens=max_tokens, temperature=0.0,
                                               ignore_eos=True)) for _ in range(n)]

    dec = add(a.decode, 200)
    while any(len(s.output_ids) < 1 for s in dec):   # their prefills, then they decode
        eng.step()
    per_step = max(1, (a.budget - a.decode) // a.prompt + 1)

    def run(n):
        for _ in range(n):
            add(per_step, 1)   # new prompts; each finishes after its first token
            eng.step()

    run(6)                                          # warm-up: shapes, graphs
    torch.cuda.synchronize()
    time.sleep(0.5)                                 # the gap the trace splitter finds
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"ms_per_mixed_step": round(dt * 1e3, 3), "decode_rows": a.decode,
                      "budget": a.budget, "new_prompts_per_step": per_step}))
    eng.shutdown()


if __name__ == "__main__":
    main()
