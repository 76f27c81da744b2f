"""Async load generator for the OpenAI-compatible server (aiohttp, installed).

The reference declares "Locust/AsyncIO load testing" (README.md:11,17; requirements.txt:34-36:
locust 2.29, aiohttp 3.10).  This client keeps ``concurrency`` streaming requests in flight
(closed loop, like a Locust user pool with zero think time) or fires them at a Poisson
``request_rate``, and measures at the client: output tokens/s, request/s, TTFT (first SSE chunk
carrying text) and inter-token latency percentiles.  Prompts can be token-id lists so the bench
needs no tokenizer files (the boxes are offline).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import time
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class ReqResult:
    ok: bool
    ttft: float = 0.0
    latency: float = 0.0
    itl: List[float] = field(default_factory=list)
    out_tokens: int = 0
    prompt_tokens: int = 0
    error: str = ""


def _pct(xs, q):
    if not xs:
        return 0.0
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))]


def summarize(results: List[ReqResult], wall: float) -> dict:
    ok = [r for r in results if r.ok]
    toks = sum(r.out_tokens for r in ok)
    ttft = [r.ttft for r in ok]
    itl = [x for r in ok for x in r.itl]
    lat = [r.latency for r in ok]
    return {
        "requests": len(results), "ok": len(ok), "errors": len(results) - len(ok),
        "wall_s": round(wall, 3),
        "output_tokens": toks,
        "output_tok_s": round(toks / wall, 1) if wall > 0 else 0.0,
        "total_tok_s": round((toks + sum(r.prompt_tokens for r in ok)) / wall, 1) if wall else 0.0,
        "req_s": round(len(ok) / wall, 3) if wall > 0 else 0.0,
        "ttft_p50_ms": round(1000 * _pct(ttft, 0.5), 2),
        "ttft_p90_ms": round(1000 * _pct(ttft, 0.9), 2),
        "ttft_p99_ms": round(1000 * _pct(ttft, 0.99), 2),
        "itl_p50_ms": round(1000 * _pct(itl, 0.5), 3),
        "itl_p90_ms": round(1000 * _pct(itl, 0.9), 3),
        "itl_p95_ms": round(1000 * _pct(itl, 0.95), 3),
        "itl_p99_ms": round(1000 * _pct(itl, 0.99), 3),
        "itl_max_ms": round(1000 * max(itl), 3) if itl else 0.0,
        "itl_mean_ms": round(1000 * sum(itl) / len(itl), 3) if itl else 0.0,
        "latency_p50_s": round(_pct(lat, 0.5), 3),
    }


async def one_request(session, url: str, prompt, max_tokens: int, model: str) -> ReqResult:
    body = {"model": model, "prompt": prompt, "max_tokens": max_tokens, "temperature": 0.0,
            "stream": True, "ignore_eos": True}
    t0 = time.perf_counter()
    first = None
    last = t0
    itl = []
    buf = b""
    done = False
    try:
        async with session.post(url + "/v1/completions", json=body) as resp:
            if resp.status != 200:
                return ReqResult(False, error=f"HTTP {resp.status}")
            # whole network chunks, split into SSE events here: one Python-level read per chunk
            # instead of three readline() calls per event (at 256 streams x ~50 events/s the
            # client's own per-event work would otherwise show up as inter-token latency); the
            # events of one chunk arrived together and share its timestamp
            async for chunk in resp.content.iter_any():
                now = time.perf_counter()
                buf += chunk
                while b"\n\n" in buf:
                    ev, buf = buf.split(b"\n\n", 1)
                    ev = ev.strip()
                    if not ev.startswith(b"data: "):
                        continue
                    if ev.startswith(b"data: [DONE]"):
                        done = True
                        break
                    if b'"choices"' not in ev:
                        j = json.loads(ev[6:])
                        return ReqResult(False, error=str(j.get("error", j)))
                    # one event per generated-token step (text may be empty)
                    if first is None:
                        first = now
                    else:
                        itl.append(now - last)
                    last = now
                if done:
                    break
    except Exception as e:  # network error -> failed request
        return ReqResult(False, error=repr(e))
    plen = len(prompt) if isinstance(prompt, list) else 0
    return ReqResult(True, (first or last) - t0, last - t0, itl, max_tokens, plen)


def _prompts(num_requests: int, prompt_len: int, vocab: int, seed: int):
    rng = random.Random(seed)
    return [[rng.randrange(3, vocab) for _ in range(prompt_len)] for _ in range(num_requests)]


async def _drive(url, prompts, concurrency, max_tokens, request_rate, model, seed):
    """Run ``prompts`` against the server; returns (results, wall seconds)."""
    import aiohttp

    rng = random.Random(seed + 1)
    results: List[ReqResult] = []
    timeout = aiohttp.ClientTimeout(total=3600)
    conn = aiohttp.TCPConnector(limit=max(concurrency, 1) + 8)
    async with aiohttp.ClientSession(timeout=timeout, connector=conn) as session:
        t0 = time.perf_counter()
        if request_rate:
            tasks = []
            for p in prompts:
                tasks.append(asyncio.create_task(one_request(session, url, p, max_tokens, model)))
                await asyncio.sleep(rng.expovariate(request_rate))
            results = list(await asyncio.gather(*tasks))
        else:
            it = iter(prompts)

            async def user():
                for p in it:
                    results.append(await one_request(session, url, p, max_tokens, model))

            await asyncio.gather(*[user() for _ in range(concurrency)])
        wall = time.perf_counter() - t0
    return results, wall


async def run_load(url: str, num_requests: int, concurrency: int, prompt_len: int,
                   max_tokens: int, vocab: int = 32000, request_rate: Optional[float] = None,
                   model: str = "lumen", seed: int = 0) -> dict:
    prompts = _prompts(num_requests, prompt_len, vocab, seed)
    results, wall = await _drive(url, prompts, concurrency, max_tokens, request_rate, model, seed)
    return summarize(results, wall)


def _worker(i, url, prompts, concurrency, max_tokens, rate, model, seed, warmup, ready, go, out):
    """One load-generator process (Locust's distributed worker): warm up, report ready, wait for
    the common start, run its share, send back raw per-request results and its end time."""
    if warmup:
        asyncio.run(_drive(url, prompts[:warmup], warmup, 4, None, model, seed))
    ready.put(i)
    go.wait()
    t0 = time.time()
    results, _ = asyncio.run(_drive(url, prompts, concurrency, max_tokens, rate, model, seed + i))
    out.put((i, t0, time.time(), [(r.ok, r.ttft, r.latency, r.itl, r.out_tokens, r.prompt_tokens,
                                    r.error) for r in results]))


def run_load_procs(url: str, num_requests: int, concurrency: int, prompt_len: int,
                   max_tokens: int, vocab: int = 32000, request_rate: Optional[float] = None,
                   model: str = "lumen", seed: int = 0, procs: int = 1, warmup: int = 0) -> dict:
    """``run_load`` spread over ``procs`` client processes (requests and concurrency split
    round-robin, one common start): at hundreds of streams a single asyncio client saturates
    its core and its own lag reads as server latency.  Wall = first start to last end."""
    import multiprocessing as mp

    prompts = _prompts(num_requests, prompt_len, vocab, seed)
    ctx = mp.get_context("spawn")
    ready, out, go = ctx.Queue(), ctx.Queue(), ctx.Event()
    ps = []
    for i in range(procs):
        share = prompts[i::procs]
        conc = len(range(i, concurrency, procs))
        rate = request_rate / procs if request_rate else None
        wu = len(range(i, warmup, procs))
        p = ctx.Process(target=_worker, args=(i, url, share, max(conc, 1), max_tokens, rate, model,
                                              seed, wu, ready, go, out), daemon=True)
        p.start()
        ps.append(p)
    def collect(q, n, limit):
        got, t0 = [], time.time()
        while len(got) < n:
            try:
                got.append(q.get(timeout=1.0))
            except Exception:  # queue.Empty: fail fast if a worker died instead of waiting
                dead = [p.exitcode for p in ps if p.exitcode not in (None, 0)]
                if dead or time.time() - t0 > limit:
                    for p in ps:
                        p.kill()
                    raise RuntimeError(f"load-client worker failed (exit codes {dead})")
        return got

    collect(ready, procs, 600)
    go.set()
    parts = collect(out, procs, 3600)
    for p in ps:
        p.join(30)
    t0 = min(x[1] for x in parts)
    t1 = max(x[2] for x in parts)
    results = [ReqResult(ok, ttft, lat, itl, n, pt, err)
               for _, _, _, rs in parts for ok, ttft, lat, itl, n, pt, err in rs]
    res = summarize(results, t1 - t0)
    res["client_procs"] = procs
    return res


def main():
    ap = argparse.ArgumentParser(description="lumen async OpenAI-API load generator")
    ap.add_argument("--url", default="http://127.0.0.1:8000")
    ap.add_argument("--num-requests", type=int, default=256)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--request-rate", type=float, default=None)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--model", default="lumen")
    ap.add_argument("--warmup", type=int, default=0,
                    help="first run this many short (4-token) requests, untimed")
    ap.add_argument("--procs", type=int, default=1,
                    help="client processes (Locust-style distributed workers)")
    a = ap.parse_args()
    if a.procs > 1:
        res = run_load_procs(a.url, a.num_requests, a.concurrency, a.prompt_len, a.max_tokens,
                             a.vocab, a.request_rate, a.model, procs=a.procs, warmup=a.warmup)
        print(json.dumps(res))
        return
    if a.warmup:
        asyncio.run(run_load(a.url, a.warmup, a.warmup, a.prompt_len, 4, a.vocab,
                             model=a.model, seed=1))
    res = asyncio.run(run_load(a.url, a.num_requests, a.concurrency, a.prompt_len, a.max_tokens,
                               a.vocab, a.request_rate, a.model))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
