"""Locust load profile for the OpenAI-compatible server (the reference declares
locust 2.29 for HTTP load tests, requirements.txt:34-36, README.md:11,17).

    locust -f lumen/bench/locustfile.py --host http://127.0.0.1:8000 \
           --users 256 --spawn-rate 32 --run-time 5m --headless

Each simulated user streams ``/v1/completions`` (or ``/v1/chat/completions`` with
``LUMEN_LOCUST_CHAT=1``) and reports time-to-first-token and whole-request latency as separate
Locust request types, so the Locust UI/CSV shows TTFT and end-to-end percentiles side by side.
Prompt/response lengths come from ``LUMEN_LOCUST_IN`` / ``LUMEN_LOCUST_OUT`` (default 512 / 128,
the serve-bench shape).  locust is not installed in this image; the module imports without it
(``HttpUser`` falls back to ``object``) so the payload logic stays unit-testable, and
``lumen.bench.async_client`` is the in-tree aiohttp equivalent used by ``serve_bench``.
"""
from __future__ import annotations

import json
import os
import random
import time

try:  # pragma: no cover - exercised only where locust is installed
    from locust import HttpUser, between, events, task
except ImportError:  # keep importable for tests / docs
    HttpUser = object
    events = None

    def between(a, b):
        return lambda *_: random.uniform(a, b)

    def task(f=None, *_a, **_k):
        return f if callable(f) else (lambda g: g)


PROMPT_TOKENS = int(os.environ.get("LUMEN_LOCUST_IN", "512"))
MAX_TOKENS = int(os.environ.get("LUMEN_LOCUST_OUT", "128"))
USE_CHAT = os.environ.get("LUMEN_LOCUST_CHAT", "0") == "1"
MODEL = os.environ.get("LUMEN_LOCUST_MODEL", "lumen")
_WORDS = ["alpha", "beta", "gamma", "delta", "kernel", "wave", "tile", "cache", "token", "graph"]


def make_prompt(n_words: int, rng: random.Random) -> str:
    return " ".join(rng.choice(_WORDS) for _ in range(n_words))


def make_payload(rng: random.Random, chat: bool = USE_CHAT, prompt_tokens: int = PROMPT_TOKENS,
                 max_tokens: int = MAX_TOKENS) -> dict:
    # ~1 token per word for the byte/BPE tokenizers used offline
    text = make_prompt(prompt_tokens, rng)
    body = {"model": MODEL, "max_tokens": max_tokens, "temperature": 0.0, "stream": True,
            "ignore_eos": True}
    if chat:
        body["messages"] = [{"role": "user", "content": text}]
    else:
        body["prompt"] = text
    return body


def parse_sse_line(line: bytes):
    """Return the decoded JSON chunk of one SSE ``data:`` line, or None (keep-alive / [DONE])."""
    if not line or not line.startswith(b"data:"):
        return None
    data = line[5:].strip()
    if data == b"[DONE]":
        return None
    return json.loads(data)


class CompletionUser(HttpUser):
    wait_time = between(0.0, 0.1)

    def on_start(self):
        self.rng = random.Random(id(self))

    @task
    def stream_completion(self):
        path = "/v1/chat/completions" if USE_CHAT else "/v1/completions"
        body = make_payload(self.rng)
        t0 = time.perf_counter()
        ttft = None
        n_chunks = 0
        with self.client.post(path, json=body, stream=True, catch_response=True,
                              name=path) as resp:
            if resp.status_code != 200:
                resp.failure(f"HTTP {resp.status_code}")
                return
            for line in resp.iter_lines():
                chunk = parse_sse_line(line)
                if chunk is None:
                    continue
                if ttft is None:
                    ttft = time.perf_counter() - t0
                n_chunks += 1
            resp.success()
        if events is not None and ttft is not None:
            events.request.fire(request_type="TTFT", name=path, response_time=ttft * 1000.0,
                                response_length=0, exception=None, context={})
            events.request.fire(request_type="TOKENS", name=path,
                                response_time=(time.perf_counter() - t0) * 1000.0,
                                response_length=n_chunks, exception=None, context={})
