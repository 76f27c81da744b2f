"""Serving benchmark: Llama-2-7B, TP=1, on one MI355X (BASELINE.json config 4).

Metric: "serve tok/s + p50 TTFT".  Two modes:
  * ``--mode engine``: in-process LLMEngine, ``--num-requests`` requests arriving all at once (or
    at ``--request-rate``), continuous batching; output tokens/s over the wall time of the run
    and TTFT = first-token time - arrival per request.
  * ``--mode http``: the production serving path -- engine core in this process, the OpenAI
    server in a spawned process, the async client (lumen.bench.async_client) in a third: the
    API + load-generator path the reference declares.
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


def make_engine(a):
    """The LLMEngine both modes serve from (Llama-2-7B preset, random init, bf16)."""
    from lumen.serve.engine import EngineConfig, LLMEngine

    cfg = EngineConfig(model=a.model, dtype="bf16", max_model_len=a.max_model_len,
                       max_num_seqs=a.max_num_seqs, max_num_batched_tokens=a.max_batched_tokens,
                       prefill_boost=a.prefill_boost, use_graphs=not a.no_graphs, init="random",
                       async_scheduling=not a.sync_scheduling, kv_cache_dtype=a.kv_cache_dtype,
                       tp_size=getattr(a, "tp", 1),
                       scheduling_policy=getattr(a, "scheduling_policy", "chunked"),
                       num_blocks=getattr(a, "num_blocks", None),
                       enable_prefix_caching=getattr(a, "enable_prefix_caching", False),
                       num_speculative_tokens=getattr(a, "num_speculative_tokens", 0))
    t0 = time.time()
    eng = LLMEngine(cfg)
    eng._bench_setup_s = time.time() - t0
    return eng


def _warm(eng, a, rng):
    """Warm-up: capture the decode-bucket graphs this run will touch."""
    import torch

    from lumen.serve.sequence import SamplingParams

    V = eng.model_config.vocab_size
    warm = [eng.add_request([rng.randrange(3, V) for _ in range(a.prompt_len)],
                            SamplingParams(max_tokens=4, temperature=0, ignore_eos=True))
            for _ in range(min(a.num_requests, a.max_num_seqs))]
    while any(not s.finished for s in warm):
        eng.step()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def bench_engine(a, eng=None) -> dict:
    import torch

    from lumen.serve.sequence import SamplingParams

    eng = eng if eng is not None else make_engine(a)
    rng = random.Random(0)
    V = eng.model_config.vocab_size
    mk = lambda n: [rng.randrange(3, V) for _ in range(n)]  # noqa: E731
    _warm(eng, a, rng)
    params = dict(max_tokens=a.max_tokens, temperature=a.temperature, ignore_eos=True)
    if getattr(a, "top_p", None) is not None:
        params["top_p"] = a.top_p
    if getattr(a, "top_k", None) is not None:
        params["top_k"] = a.top_k
    # --shared-prefix N: every prompt starts with the same N tokens (a shared system prompt)
    shared = mk(min(getattr(a, "shared_prefix", 0), a.prompt_len))
    prompts = [shared + mk(a.prompt_len - len(shared)) for _ in range(a.num_requests)]
    hit0, q0, pf0 = eng.blocks.hit_tokens, eng.blocks.query_tokens, eng.stats["prefill_tokens"]
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
        if getattr(a, "trace_steps", False):
            trace = _trace_steps(eng)
        else:
            while eng.has_work:
                eng.step()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    out_toks = sum(len(s.output_ids) for s in seqs)
    ttft = [s.first_token_time - s.arrival for s in seqs]
    itl = [b - a_ for s in seqs for a_, b in zip(s.token_times, s.token_times[1:])]
    extra = {"step_trace": trace} if getattr(a, "trace_steps", False) else {}
    return {**extra, "mode": "engine", "requests": len(seqs), "prompt_len": a.prompt_len,
            "max_tokens": a.max_tokens, "wall_s": round(wall, 3), "output_tokens": out_toks,
            "output_tok_s": round(out_toks / wall, 1),
            "total_tok_s": round((out_toks + a.prompt_len * len(seqs)) / wall, 1),
            "ttft_p50_ms": round(1000 * _pct(ttft, 0.5), 2),
            "ttft_p99_ms": round(1000 * _pct(ttft, 0.99), 2),
            "itl_p50_ms": round(1000 * _pct(itl, 0.5), 3),
            "itl_p99_ms": round(1000 * _pct(itl, 0.99), 3),
            "itl_max_ms": round(1000 * max(itl), 3) if itl else 0.0,
            "itl_mean_ms": round(1000 * sum(itl) / len(itl), 3) if itl else 0.0,
            "scheduling_policy": getattr(a, "scheduling_policy", "chunked"),
            "kv_blocks": eng.blocks.num_blocks, "preemptions": eng.scheduler.num_preemptions,
            "max_batched_tokens": a.max_batched_tokens, "steps": eng.stats["steps"],
            "async_scheduling": eng.async_sched, "kv_cache_dtype": a.kv_cache_dtype,
            "setup_s": round(getattr(eng, "_bench_setup_s", 0.0), 1),
            "graphs": sorted(eng.runner._graphs),
            "shared_prefix": len(shared), "prefix_caching": eng.blocks.prefix_caching,
            "prefix_hit_rate": round((eng.blocks.hit_tokens - hit0)
                                     / max(1, eng.blocks.query_tokens - q0), 4),
            "prefill_tokens_computed": eng.stats["prefill_tokens"] - pf0,
            "spec": {k: eng.stats[k] for k in ("spec_steps", "spec_proposed", "spec_accepted")}}


def _trace_steps(eng) -> dict:
    """Drive the engine to completion timing every step on the device clock (synchronous: each
    step is waited for), grouped by composition: decode-only, prefill-only and mixed steps with
    their mean prefill tokens / decode rows -- where a scheduling policy's time goes."""
    import torch

    kinds = {}
    orig = eng.scheduler.schedule
    last = {}

    def spy():
        b = orig()
        if b is not None:
            last["p"] = sum(c for _, c in b.prefills)
            last["d"] = len(b.decodes)
        return b

    eng.scheduler.schedule = spy
    try:
        while eng.has_work:
            last.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if not last:
                continue
            k = "mixed" if last["p"] and last["d"] else ("prefill" if last["p"] else "decode")
            g = kinds.setdefault(k, [0, 0.0, 0, 0])
            g[0] += 1
            g[1] += dt
            g[2] += last["p"]
            g[3] += last["d"]
    finally:
        eng.scheduler.schedule = orig
    return {k: {"steps": n, "ms_total": round(1000 * t, 1), "ms_mean": round(1000 * t / n, 2),
                "prefill_tokens_mean": round(p / n, 1), "decode_rows_mean": round(d / n, 1)}
            for k, (n, t, p, d) in kinds.items()}


def bench_http(a, eng=None) -> dict:
    """The production serving path (``scripts/serve.py``): the engine core loop in THIS (GPU)
    process, the OpenAI HTTP server in ``a.api_servers`` spawned processes talking to it over
    queues (one port, SO_REUSEPORT), and the async client (the Locust request shape: streamed
    ``/v1/completions`` with ``ignore_eos``) in ``a.client_procs`` more processes (Locust's
    distributed workers) -- neither the front-end's nor the client's per-event Python work
    competes with the engine for a GIL or saturates a core.  With ``eng`` (already warm, e.g.
    after ``bench_engine``) no model load or graph capture is paid again."""
    import threading
    import urllib.request

    from lumen.serve.frontend import run_engine_core, start_api_servers

    t0 = time.time()
    eng = eng if eng is not None else make_engine(a)
    n_api = int(getattr(a, "api_servers", 1))
    n_cli = int(getattr(a, "client_procs", 1))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    url = f"http://127.0.0.1:{port}"
    req_q, out_qs, apis = start_api_servers(n_api, a.model, a.max_model_len, "127.0.0.1", port,
                                            "lumen", eng.model_config.vocab_size)
    client = None
    try:
        while True:
            try:
                urllib.request.urlopen(url + "/health", timeout=2)
                break
            except Exception:
                if not all(p.is_alive() for p in apis) or time.time() - t0 > 300:
                    raise RuntimeError("API server did not come up")
                time.sleep(0.2)
        cmd = [sys.executable, "-m", "lumen.bench.async_client", "--url", url,
               "--num-requests", str(a.num_requests), "--concurrency", str(a.concurrency),
               "--prompt-len", str(a.prompt_len), "--max-tokens", str(a.max_tokens),
               "--vocab", str(eng.model_config.vocab_size),
               "--warmup", str(min(a.concurrency, a.num_requests)), "--procs", str(n_cli)]
        if a.request_rate:
            cmd += ["--request-rate", str(a.request_rate)]
        client = subprocess.Popen(cmd, stdout=subprocess.PIPE, cwd=ROOT,
                                  env=dict(os.environ, PYTHONPATH=ROOT))
        out = {}

        def watch():  # the engine core loop ends when the client has its numbers
            out["stdout"] = client.communicate()[0]
            req_q.put(("stop",))

        w = threading.Thread(target=watch, daemon=True)
        w.start()
        run_engine_core(eng, req_q, out_qs)
        w.join()
        if client.returncode != 0:
            raise RuntimeError(f"load client exited with {client.returncode}")
        lines = [x for x in out["stdout"].decode().splitlines() if x.startswith("{")]
        res = json.loads(lines[-1])
    finally:
        for q in out_qs:
            q.put(None)
        if client is not None and client.poll() is None:
            client.kill()
        for p in apis:
            p.terminate()
        for p in apis:
            p.join(10)
    res["mode"] = "http"
    # leak check: every request finished, every KV block back (prefix-cached ones parked)
    res["kv_blocks"], res["kv_blocks_free_at_end"] = eng.blocks.num_blocks, eng.blocks.num_free
    res["engine_requests_left"] = len(eng.scheduler.running) + len(eng.scheduler.waiting)
    res["prefix_hit_rate"] = round(eng.blocks.hit_rate, 4)
    res["api_servers"], res["client_procs"] = n_api, n_cli
    res["prompt_len"], res["max_tokens"] = a.prompt_len, a.max_tokens
    res["http_section_s"] = round(time.time() - t0, 1)
    return res


def main():
    sys.path.insert(0, ROOT)
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="engine", choices=["engine", "http", "both"])
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--num-requests", type=int, default=256)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--request-rate", type=float, default=None)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top-p", type=float, default=None)
    ap.add_argument("--top-k", type=int, default=None)
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=2048)
    ap.add_argument("--prefill-boost", type=int, default=1,
                    help="x token budget while at most max-num-seqs/4 sequences decode (1: off)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    ap.add_argument("--sync-scheduling", action="store_true",
                    help="engine mode: host waits for each step's tokens before the next step")
    ap.add_argument("--tp", type=int, default=1,
                    help="engine mode, under torch.distributed.run: tensor-parallel degree; rank 0 "
                         "runs the bench, the other ranks the worker loop")
    ap.add_argument("--num-blocks", type=int, default=None, help="KV blocks (default: auto)")
    ap.add_argument("--scheduling-policy", default="chunked", choices=["chunked", "prefill_first"])
    ap.add_argument("--enable-prefix-caching", action="store_true")
    ap.add_argument("--num-speculative-tokens", type=int, default=0,
                    help="prompt-lookup speculative decoding (greedy requests)")
    ap.add_argument("--shared-prefix", type=int, default=0,
                    help="engine mode: the first N prompt tokens are the same in every request")
    ap.add_argument("--api-servers", type=int, default=1,
                    help="http mode: OpenAI API processes sharing the port (SO_REUSEPORT)")
    ap.add_argument("--client-procs", type=int, default=1,
                    help="http mode: load-client processes (Locust-style workers)")
    ap.add_argument("--trace-steps", action="store_true",
                    help="engine mode: time every step synchronously, grouped by composition")
    a = ap.parse_args()
    if a.tp > 1:
        from lumen.parallel.dist import init, shutdown

        env = init()
        if env.world_size != a.tp:
            raise SystemExit(f"--tp {a.tp} but WORLD_SIZE={env.world_size}")
        eng = make_engine(a)
        if env.rank != 0:
            from lumen.serve.tp import worker_loop

            worker_loop(eng.runner)
            shutdown()
            return
        res = bench_engine(a, eng)
        eng.shutdown()
        res.update(metric="serve tok/s + p50 TTFT", model=a.model, tp=a.tp, dtype="bf16",
                   data="random token-id prompts; random-init weights")
        print(json.dumps(res), flush=True)
        shutdown()
        return
    if a.mode == "both":
        eng = make_engine(a)
        res = bench_http(a, eng)
        res["engine"] = bench_engine(a, eng)
    else:
        res = bench_engine(a) if a.mode == "engine" else bench_http(a)
    res.update(metric="serve tok/s + p50 TTFT (Llama-2-7B, TP=1)", model=a.model, dtype="bf16",
               data="random token-id prompts; random-init weights")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
