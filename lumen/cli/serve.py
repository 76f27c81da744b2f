"""``python -m lumen.cli.serve`` / ``scripts/serve.py``: OpenAI-compatible server.

    python scripts/serve.py --model meta-llama/Llama-2-7b-hf --adapter checkpoints/x/final
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 scripts/serve.py --tp 2 ...

Rank 0 runs the scheduler + HTTP server; under TP the other ranks run the worker loop.
"""
from __future__ import annotations

import argparse
import os
import sys


def resolve_scheduling(policy, enable_chunked_prefill, budget, max_model_len):
    """(policy, tokens per step) with vLLM 0.6.0's defaults (the version the reference pins,
    requirements.txt:18): chunked prefill off -- prefill-only steps while prompts wait, at most
    max(max_model_len, 2048) tokens per step; ``--enable-chunked-prefill`` = mixed steps."""
    if policy is None:
        policy = "chunked" if enable_chunked_prefill else "prefill_first"
    elif enable_chunked_prefill and policy != "chunked":
        raise SystemExit("--enable-chunked-prefill contradicts --scheduling-policy " + policy)
    if budget is None:
        budget = max(max_model_len, 2048) if policy == "prefill_first" else 2048
    return policy, budget


def build_parser():
    ap = argparse.ArgumentParser(description="lumen OpenAI-compatible server (MI355X)")
    ap.add_argument("--model", default="meta-llama/Llama-2-7b-hf",
                    help="preset / hub id (random init offline) or local HF checkpoint dir")
    ap.add_argument("--adapter", "--lora", default=None, help="PEFT LoRA adapter dir to merge")
    ap.add_argument("--lora-modules", nargs="*", default=None, metavar="NAME=PATH",
                    help="serve these PEFT adapters un-merged; requests pick one with 'model'")
    ap.add_argument("--max-loras", type=int, default=4)
    ap.add_argument("--served-model-name", default=None)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--tp", "--tensor-parallel-size", "--tensor_parallel_size", type=int, default=1, help="tensor-parallel degree (= world size)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=None,
                    help="tokens per engine step; default as vLLM 0.6.0: max(max-model-len, 2048) "
                         "for prefill_first, 2048 for chunked")
    ap.add_argument("--prefill-boost", type=int, default=1,
                    help="x token budget while at most max-num-seqs/4 sequences decode (1: off)")
    ap.add_argument("--enable-chunked-prefill", action="store_true",
                    help="vLLM's flag: same as --scheduling-policy chunked")
    ap.add_argument("--scheduling-policy", default=None, choices=["chunked", "prefill_first"],
                    help="prefill_first (default, vLLM 0.6.0's: prefill-only steps while prompts "
                         "wait, then decode steps); chunked: mixed prefill-chunk + decode steps "
                         "(bounded inter-token latency)")
    ap.add_argument("--block-size", type=int, default=16)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.9)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="KV-cache element type (fp8 = e4m3: 2x capacity, half the decode K/V reads)")
    ap.add_argument("--enable-prefix-caching", action="store_true",
                    help="share the cached K/V of equal leading prompt blocks across requests "
                         "(vLLM's flag; finished requests' blocks stay cached until evicted)")
    ap.add_argument("--speculative-model", default=None,
                    help='"[ngram]": speculative decoding by prompt lookup (the only drafter)')
    ap.add_argument("--num-speculative-tokens", type=int, default=0,
                    help="draft tokens per step with --speculative-model [ngram]")
    ap.add_argument("--ngram-prompt-lookup-max", type=int, default=4)
    ap.add_argument("--ngram-prompt-lookup-min", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--api-server-count", type=int, default=1,
                    help="OpenAI API processes sharing --port (SO_REUSEPORT), each streaming its "
                         "own requests' tokens from the one engine core")
    ap.add_argument("--in-process", action="store_true",
                    help="run the HTTP server on a thread of the GPU process (default: the API "
                         "runs in its own process and talks to the engine core over queues)")
    return ap


def main(argv=None):
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, root)
    a = build_parser().parse_args(argv)
    from lumen.models import get_config

    rank = int(os.environ.get("RANK", "0"))
    apis, req_q, out_qs = [], None, []
    if rank == 0 and not a.in_process:
        # OpenAI HTTP front-end(s) in spawned processes (no GPU, their own GILs), started before
        # this process initialises the GPU; they talk to the engine core below over queues
        from lumen.serve.frontend import start_api_servers

        mcfg = get_config(a.model)
        lora_names = [m.split("=", 1)[0] for m in (a.lora_modules or [])]
        req_q, out_qs, apis = start_api_servers(a.api_server_count, a.model, a.max_model_len,
                                                a.host, a.port, a.served_model_name,
                                                mcfg.vocab_size, lora_names)

    from lumen.parallel.dist import init
    from lumen.serve.engine import AsyncEngine, EngineConfig, LLMEngine

    env = init()
    if env.world_size != a.tp:
        raise SystemExit(f"--tp {a.tp} but WORLD_SIZE={env.world_size}")
    if a.speculative_model not in (None, "[ngram]"):
        raise SystemExit('--speculative-model: only "[ngram]" (prompt lookup) is served')
    spec_k = a.num_speculative_tokens if a.speculative_model == "[ngram]" else 0
    policy, budget = resolve_scheduling(a.scheduling_policy, a.enable_chunked_prefill,
                                        a.max_num_batched_tokens, a.max_model_len)
    cfg = EngineConfig(model=a.model, adapter=a.adapter, dtype=a.dtype,
                       max_model_len=a.max_model_len, block_size=a.block_size,
                       gpu_memory_utilization=a.gpu_memory_utilization,
                       max_num_seqs=a.max_num_seqs, max_num_batched_tokens=budget,
                       prefill_boost=a.prefill_boost, tp_size=a.tp, seed=a.seed, use_graphs=not a.no_graphs,
                       scheduling_policy=policy,
                       kv_cache_dtype=a.kv_cache_dtype,
                       enable_prefix_caching=a.enable_prefix_caching,
                       num_speculative_tokens=spec_k,
                       ngram_max=a.ngram_prompt_lookup_max, ngram_min=a.ngram_prompt_lookup_min,
                       lora_modules=dict(m.split("=", 1) for m in a.lora_modules)
                       if a.lora_modules else None, max_loras=a.max_loras)
    eng = LLMEngine(cfg)
    if env.rank != 0:
        from lumen.serve.tp import worker_loop

        worker_loop(eng.runner)
        return
    print(f"[lumen.serve] {cfg.model} tp={a.tp} kv_blocks={eng.blocks.num_blocks} "
          f"on http://{a.host}:{a.port}", flush=True)
    if a.in_process:
        import uvicorn

        from lumen.serve.api_server import create_app

        app = create_app(AsyncEngine(eng), a.served_model_name)
        try:
            uvicorn.run(app, host=a.host, port=a.port, log_level="warning")
        finally:
            eng.shutdown()
        return
    import signal

    from lumen.serve.frontend import run_engine_core

    def _term(signum, frame):  # SIGTERM -> unwind through finally: stop the API process too
        raise SystemExit(0)

    signal.signal(signal.SIGTERM, _term)
    try:
        run_engine_core(eng, req_q, out_qs)
    except KeyboardInterrupt:
        pass
    finally:
        for q in out_qs:
            q.put(None)
        for p in apis:
            p.terminate()
        for p in apis:
            p.join(10)
        eng.shutdown()


if __name__ == "__main__":
    main()
