"""Serving benchmark: Llama-2-7B, TP=1, on one MI355X (BASELINE.json config 4).

Metric: "serve tok/s + p50 TTFT".  Two modes:
  * ``--mode engine``: in-process LLMEngine, ``--num-requests`` requests arriving all at once (or
    at ``--request-rate``), continuous batching; output tokens/s over the wall time of the run
    and TTFT = first-token time - arrival per request.
  * ``--mode http``: starts the OpenAI server in a subprocess and drives it with the async
    client (lumen.bench.async_client) -- the API + load-generator path the reference declares.
Random-init weights, random token-id prompts (offline); ``ignore_eos`` so every request produces
exactly ``--max-tokens`` tokens.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))] if s else 0.0


def bench_engine(a) -> dict:
    import torch

    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    cfg = EngineConfig(model=a.model, dtype="bf16", max_model_len=a.max_model_len,
                       max_num_seqs=a.max_num_seqs, max_num_batched_tokens=a.max_batched_tokens,
                       prefill_boost=a.prefill_boost, use_graphs=not a.no_graphs, init="random",
                       async_scheduling=not a.sync_scheduling, kv_cache_dtype=a.kv_cache_dtype)
    t0 = time.time()
    eng = LLMEngine(cfg)
    setup = time.time() - t0
    rng = random.Random(0)
    V = eng.model_config.vocab_size
    mk = lambda n: [rng.randrange(3, V) for _ in range(n)]  # noqa: E731
    # warm-up: compile graphs for the decode buckets this run will touch
    warm = [eng.add_request(mk(a.prompt_len), SamplingParams(max_tokens=4, temperature=0,
                                                              ignore_eos=True))
            for _ in range(min(a.num_requests, a.max_num_seqs))]
    while any(not s.finished for s in warm):
        eng.step()
    torch.cuda.synchronize()
    params = dict(max_tokens=a.max_tokens, temperature=a.temperature, ignore_eos=True)
    prompts = [mk(a.prompt_len) for _ in range(a.num_requests)]
    seqs = []
    t_start = time.perf_counter()
    if a.request_rate:
        next_t = t_start
        pending = list(prompts)
        while pending or eng.has_work:
            now = time.perf_counter()
            while pending and now >= next_t:
                seqs.append(eng.add_request(pending.pop(0), SamplingParams(**params)))
                next_t += rng.expovariate(a.request_rate)
            if eng.has_work:
                eng.step()
            else:
                time.sleep(max(0.0, next_t - time.perf_counter()))
    else:
        seqs = [eng.add_request(p, SamplingParams(**params)) for p in prompts]
        while eng.has_work:
            eng.step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    out_toks = sum(len(s.output_ids) for s in seqs)
    ttft = [s.first_token_time - s.arrival for s in seqs]
    itl = [b - a_ for s in seqs for a_, b in zip(s.token_times, s.token_times[1:])]
    return {"mode": "engine", "requests": len(seqs), "prompt_len": a.prompt_len,
            "max_tokens": a.max_tokens, "wall_s": round(wall, 3), "output_tokens": out_toks,
            "output_tok_s": round(out_toks / wall, 1),
            "total_tok_s": round((out_toks + a.prompt_len * len(seqs)) / wall, 1),
            "ttft_p50_ms": round(1000 * _pct(ttft, 0.5), 2),
            "ttft_p99_ms": round(1000 * _pct(ttft, 0.99), 2),
            "itl_p50_ms": round(1000 * _pct(itl, 0.5), 3),
            "itl_p99_ms": round(1000 * _pct(itl, 0.99), 3),
            "kv_blocks": eng.blocks.num_blocks, "preemptions": eng.scheduler.num_preemptions,
            "max_batched_tokens": a.max_batched_tokens, "steps": eng.stats["steps"],
            "async_scheduling": eng.async_sched, "kv_cache_dtype": a.kv_cache_dtype,
            "setup_s": round(setup, 1), "graphs": sorted(eng.runner._graphs)}


def bench_http(a) -> dict:
    from lumen.bench.async_client import run_load

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "serve.py"), "--model", a.model,
           "--port", str(port), "--max-model-len", str(a.max_model_len),
           "--max-num-seqs", str(a.max_num_seqs),
           "--max-num-batched-tokens", str(a.max_batched_tokens),
           "--prefill-boost", str(a.prefill_boost)]
    if a.no_graphs:
        cmd.append("--no-graphs")
    if a.kv_cache_dtype != "auto":
        cmd += ["--kv-cache-dtype", a.kv_cache_dtype]
    proc = subprocess.Popen(cmd, env=dict(os.environ, PYTHONPATH=ROOT))
    url = f"http://127.0.0.1:{port}"
    try:
        import urllib.request

        t0 = time.time()
        while True:
            try:
                urllib.request.urlopen(url + "/health", timeout=2)
                break
            except Exception:
                if proc.poll() is not None or time.time() - t0 > 600:
                    raise RuntimeError("server did not come up")
                time.sleep(1)
        # warm-up round (graph capture for the buckets)
        asyncio.run(run_load(url, min(a.concurrency, a.num_requests), a.concurrency,
                             a.prompt_len, 4))
        res = asyncio.run(run_load(url, a.num_requests, a.concurrency, a.prompt_len,
                                   a.max_tokens, request_rate=a.request_rate))
        res["mode"] = "http"
        res["prompt_len"], res["max_tokens"] = a.prompt_len, a.max_tokens
        return res
    finally:
        proc.terminate()
        try:
            proc.wait(30)
        except subprocess.TimeoutExpired:
            proc.kill()


def main():
    sys.path.insert(0, ROOT)
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="engine", choices=["engine", "http"])
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--num-requests", type=int, default=256)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--request-rate", type=float, default=None)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=2048)
    ap.add_argument("--prefill-boost", type=int, default=1,
                    help="x token budget while at most max-num-seqs/4 sequences decode (1: off)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    ap.add_argument("--sync-scheduling", action="store_true",
                    help="engine mode: host waits for each step's tokens before the next step")
    a = ap.parse_args()
    res = bench_engine(a) if a.mode == "engine" else bench_http(a)
    res.update(metric="serve tok/s + p50 TTFT (Llama-2-7B, TP=1)", model=a.model, dtype="bf16",
               data="random token-id prompts; random-init weights")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
