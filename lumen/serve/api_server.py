"""OpenAI-compatible HTTP API (FastAPI + uvicorn, both installed) over ``AsyncEngine``.

The reference declares "vLLM ... OpenAI-compatible API" (README.md:10,16): this serves the same
surface -- ``GET /v1/models``, ``POST /v1/completions``, ``POST /v1/chat/completions`` (both with
``stream: true`` Server-Sent Events ending in ``data: [DONE]``; ``stop`` strings, ``n`` /
``best_of``, ``presence_penalty`` / ``frequency_penalty`` and vLLM's ``repetition_penalty``,
``stop_token_ids``, ``ignore_eos``, ``seed``), ``GET /health`` and a
Prometheus-format ``GET /metrics`` (requests, tokens, TTFT / inter-token latency summaries,
KV-cache usage).  Chat requests use the Llama-2 chat template the reference trains with
(``<s>[INST] {user} [/INST]``, scripts/prepare_dataset.py:12-25).
"""
from __future__ import annotations

import asyncio
import json
import time
import uuid
from typing import Any, Dict, List, Optional, Union

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

from .sequence import SamplingParams


def llama2_chat_prompt(messages: List[Dict[str, str]]) -> str:
    """Llama-2 chat format; system prompt folded into the first user turn."""
    sys_txt = ""
    out = []
    turns = [m for m in messages if m.get("role") != "system"]
    for m in messages:
        if m.get("role") == "system":
            sys_txt = f"<<SYS>>\n{m.get('content', '')}\n<</SYS>>\n\n"
    i = 0
    while i < len(turns):
        u = turns[i]
        content = u.get("content", "")
        if i == 0 and sys_txt:
            content = sys_txt + content
        if u.get("role") == "user":
            seg = f"[INST] {content} [/INST]"
            if i + 1 < len(turns) and turns[i + 1].get("role") == "assistant":
                seg += f" {turns[i + 1].get('content', '')} </s><s>"
                i += 1
            out.append(seg)
        i += 1
    return "".join(out)


class _Stats:
    def __init__(self):
        self.requests = 0
        self.errors = 0
        self.prompt_tokens = 0
        self.completion_tokens = 0
        self.ttft: List[float] = []
        self.itl: List[float] = []

    def observe(self, seq):
        self.prompt_tokens += len(seq.prompt_ids)
        self.completion_tokens += len(seq.output_ids)
        if seq.first_token_time is not None:
            self.ttft.append(seq.first_token_time - seq.arrival)
        tt = seq.token_times
        self.itl.extend(b - a for a, b in zip(tt, tt[1:]))
        self.ttft = self.ttft[-10000:]
        self.itl = self.itl[-100000:]


def _quantiles(xs, qs=(0.5, 0.9, 0.99)):
    if not xs:
        return {q: 0.0 for q in qs}
    s = sorted(xs)
    return {q: s[min(len(s) - 1, int(q * len(s)))] for q in qs}


def _params(body: Dict[str, Any], eos: Optional[int]) -> SamplingParams:
    stop_ids = body.get("stop_token_ids") or []
    return SamplingParams(max_tokens=int(body.get("max_tokens") or 16),
                          temperature=float(body.get("temperature", 1.0)),
                          top_p=float(body.get("top_p", 1.0)), top_k=int(body.get("top_k", 0) or 0),
                          stop_token_ids=list(stop_ids), ignore_eos=bool(body.get("ignore_eos", False)),
                          seed=body.get("seed"),
                          presence_penalty=float(body.get("presence_penalty") or 0.0),
                          frequency_penalty=float(body.get("frequency_penalty") or 0.0),
                          repetition_penalty=float(body.get("repetition_penalty") or 1.0))


def _logprob_request(body: Dict[str, Any], chat: bool, params: SamplingParams) -> bool:
    """OpenAI logprobs fields onto ``params``; returns whether the response carries logprobs.
    Completions: ``logprobs: k`` (the chosen token + the k most likely, 0 <= k <= 20) and
    ``echo`` (the prompt is scored too).  Chat: ``logprobs: true`` + ``top_logprobs: k``."""
    if chat:
        if not body.get("logprobs"):
            return False
        k = int(body.get("top_logprobs") or 0)
    else:
        lp = body.get("logprobs")
        if lp is None or lp is False:
            return False
        k = int(lp)
        if body.get("echo"):
            params.prompt_logprobs = k
    if not 0 <= k <= 20:
        raise ValueError("top logprobs must be in [0, 20]")
    params.logprobs = True
    params.top_logprobs = k
    return True


def completion_logprobs(decode, ids: List[int], lps: List[Optional[float]],
                        tops: List[Optional[list]], offset: int = 0) -> Dict[str, Any]:
    """OpenAI completions ``logprobs`` object: tokens, token_logprobs, top_logprobs (the
    alternatives plus the chosen token, None where a token has no score: the first prompt
    token) and text_offset (character offsets from ``offset``)."""
    toks = [decode([t]) for t in ids]
    top_out, offs = [], []
    for i, (t, lp, alt) in enumerate(zip(toks, lps, tops)):
        if lp is None:
            top_out.append(None)
        else:
            # token strings can collide (byte-fallback pieces): a key keeps its best score
            d: Dict[str, float] = {}
            for a, v in list(alt or []) + [(None, lp)]:
                key = t if a is None else decode([a])
                d[key] = max(d.get(key, v), v)
            top_out.append(d)
        offs.append(offset)
        offset += len(t)
    return {"tokens": toks, "token_logprobs": list(lps), "top_logprobs": top_out,
            "text_offset": offs}


def chat_logprobs(decode, ids: List[int], lps: List[float], tops: List[Optional[list]]):
    """OpenAI chat ``logprobs`` object: {"content": [{token, logprob, bytes, top_logprobs}]}."""
    def ent(t, lp):
        s = decode([t])
        return {"token": s, "logprob": lp, "bytes": list(s.encode("utf-8"))}
    return {"content": [dict(ent(t, lp), top_logprobs=[ent(a, v) for a, v in (alt or [])])
                        for t, lp, alt in zip(ids, lps, tops)]}


def _stops(body: Dict[str, Any]) -> List[str]:
    st = body.get("stop")
    if st is None:
        return []
    if isinstance(st, str):
        st = [st]
    if not isinstance(st, list) or not all(isinstance(x, str) for x in st) or len(st) > 16:
        raise ValueError("stop must be a string or a list of up to 16 strings")
    return [x for x in st if x]


def _n_best_of(body: Dict[str, Any], stream: bool):
    n = int(body.get("n") or 1)
    best_of = int(body.get("best_of") or n)
    if n < 1 or best_of < n or best_of > 16:
        raise ValueError("need 1 <= n <= best_of <= 16")
    if stream and best_of != n:
        raise ValueError("best_of != n cannot be streamed")
    return n, best_of


class StopChecker:
    """OpenAI ``stop`` strings over the streamed text: text that could still be the start of a
    stop string is held back (len(longest stop) - 1 characters); when one appears the output is
    cut before it (vLLM ``include_stop_str_in_output`` keeps it) and the request finishes with
    ``finish_reason: "stop"`` -- the caller then leaves the engine stream, which aborts the
    request and frees its KV blocks."""

    def __init__(self, stops: List[str], include: bool = False):
        self.stops = stops
        self.include = include
        self.hold = max((len(x) for x in stops), default=1) - 1
        self.text = ""
        self.emitted = 0
        self.stopped = False

    def feed(self, delta: str, final: bool = False) -> str:
        """Add decoded text; returns what may be sent now."""
        if self.stopped:
            return ""
        start = max(0, len(self.text) - self.hold)
        self.text += delta
        if self.stops:
            hits = [(i, x) for x in self.stops for i in [self.text.find(x, start)] if i >= 0]
            if hits:
                i, x = min(hits)
                self.text = self.text[:i + (len(x) if self.include else 0)]
                self.stopped = True
                final = True
        end = len(self.text) if final else max(self.emitted, len(self.text) - self.hold)
        out = self.text[self.emitted:end]
        self.emitted = end
        return out


class IncrementalDetokenizer:
    """Streaming text deltas in O(window) per token (re-decoding the whole output every token
    is O(n^2) per stream).  Holds back output while the last piece decodes to an incomplete
    UTF-8 / merge sequence (U+FFFD), like vLLM's prefix/read-offset scheme."""

    def __init__(self, tok):
        self.tok = tok
        self.prefix = 0
        self.read = 0
        self._prefix_text = ""   # decode(ids[prefix:read]), kept across steps (one decode/token)

    # tokens that decode to no text at all (specials, ids outside a byte-level vocabulary) would
    # otherwise keep the window growing: after this many, the window restarts past them
    MAX_SILENT = 4
    # a U+FFFD still open after this many tokens is an invalid sequence, not an incomplete one
    # (UTF-8 needs at most 4 bytes): it is emitted as is
    MAX_HELD = 16

    def step(self, ids: List[int]) -> str:
        prefix_text = self._prefix_text
        new_text = self.tok.decode(ids[self.prefix:])
        if len(new_text) > len(prefix_text) and (not new_text.endswith("\ufffd")
                                                 or len(ids) - self.read >= self.MAX_HELD):
            self.prefix, self.read = self.read, len(ids)
            self._prefix_text = self.tok.decode(ids[self.prefix:self.read])
            return new_text[len(prefix_text):]
        if (new_text == prefix_text and len(ids) - self.read >= self.MAX_SILENT
                and not new_text.endswith("\ufffd")):
            self.prefix = self.read = len(ids)
            self._prefix_text = ""
        return ""

    def flush(self, ids: List[int]) -> str:
        return self.tok.decode(ids[self.prefix:])[len(self.tok.decode(ids[self.prefix:self.read])):]


def stream_chunk(rid: str, chat: bool, created: int, model: str, delta_text: str,
                 finish: Optional[str], index: int = 0, logprobs=None) -> Dict[str, Any]:
    """One OpenAI streaming chunk (``chat.completion.chunk`` / ``text_completion``)."""
    if chat:
        d = {"content": delta_text} if delta_text else {}
        ch = {"index": index, "delta": d, "finish_reason": finish}
        if logprobs is not None:
            ch["logprobs"] = logprobs
        o = "chat.completion.chunk"
    else:
        ch = {"index": index, "text": delta_text, "logprobs": logprobs, "finish_reason": finish}
        o = "text_completion"
    return {"id": rid, "object": o, "created": created, "model": model, "choices": [ch]}


def sse_head(rid: str, chat: bool, created: int, model: str) -> str:
    """The constant part of a stream's chunks, serialised once per request."""
    return json.dumps({"id": rid, "object": "chat.completion.chunk" if chat else
                       "text_completion", "created": created, "model": model})[:-1]


def sse_event(head: str, chat: bool, delta_text: str, finish: Optional[str],
              index: int = 0) -> str:
    """``data: <json.dumps(stream_chunk(...))>`` built from the pre-serialised head: at 256
    concurrent streams the API process formats ~13k events per second, and a nested-dict dumps
    per event was a visible share of its time."""
    f = "null" if finish is None else json.dumps(finish)
    if chat:
        d = '{"content": %s}' % json.dumps(delta_text) if delta_text else "{}"
        ch = '{"index": %d, "delta": %s, "finish_reason": %s}' % (index, d, f)
    else:
        ch = ('{"index": %d, "text": %s, "logprobs": null, "finish_reason": %s}'
              % (index, json.dumps(delta_text), f))
    return 'data: %s, "choices": [%s]}\n\n' % (head, ch)


def create_app(aengine, served_model_name: Optional[str] = None):
    """``aengine``: ``AsyncEngine`` (engine thread in this process) or
    ``frontend.EngineCoreClient`` (engine core in the GPU process)."""
    name = served_model_name or aengine.model_name
    tok = aengine.tokenizer
    stats = _Stats()
    app = FastAPI(title="lumen OpenAI-compatible server")

    def decode(ids):
        return tok.decode(ids)

    @app.get("/health")
    async def health():
        return {"status": "ok"}

    @app.get("/version")
    async def version():
        import lumen
        return {"version": getattr(lumen, "__version__", "0")}

    @app.post("/tokenize")
    async def tokenize(req: Request):
        """vLLM's /tokenize: {"prompt"} or chat {"messages"} -> token ids and count."""
        body = await req.json()
        if body.get("messages"):
            text = llama2_chat_prompt(body["messages"])
        else:
            text = body.get("prompt", "")
        if not isinstance(text, str):
            raise HTTPException(status_code=400, detail="prompt must be a string")
        ids = tok.encode(text)
        return {"tokens": ids, "count": len(ids), "max_model_len": aengine.max_model_len}

    @app.post("/detokenize")
    async def detokenize(req: Request):
        body = await req.json()
        ids = body.get("tokens")
        if not isinstance(ids, list) or not all(isinstance(t, int) for t in ids):
            raise HTTPException(status_code=400, detail="tokens must be a list of ints")
        return {"prompt": decode(ids)}

    loras = list(getattr(aengine, "lora_names", []) or [])

    @app.get("/v1/models")
    async def models():
        now = int(time.time())
        data = [{"id": name, "object": "model", "created": now, "owned_by": "lumen",
                 "max_model_len": aengine.max_model_len}]
        data += [{"id": n, "object": "model", "created": now, "owned_by": "lumen", "root": name,
                  "parent": name, "max_model_len": aengine.max_model_len} for n in loras]
        return {"object": "list", "data": data}

    @app.get("/metrics")
    async def metrics():
        t, i = _quantiles(stats.ttft), _quantiles(stats.itl)
        live = aengine.live_stats()
        lines = [
            "# TYPE lumen_requests_total counter", f"lumen_requests_total {stats.requests}",
            "# TYPE lumen_request_errors_total counter", f"lumen_request_errors_total {stats.errors}",
            "# TYPE lumen_prompt_tokens_total counter", f"lumen_prompt_tokens_total {stats.prompt_tokens}",
            "# TYPE lumen_generation_tokens_total counter",
            f"lumen_generation_tokens_total {stats.completion_tokens}",
            "# TYPE lumen_time_to_first_token_seconds summary",
            *[f'lumen_time_to_first_token_seconds{{quantile="{q}"}} {v:.6f}' for q, v in t.items()],
            "# TYPE lumen_inter_token_latency_seconds summary",
            *[f'lumen_inter_token_latency_seconds{{quantile="{q}"}} {v:.6f}' for q, v in i.items()],
            "# TYPE lumen_kv_cache_usage_ratio gauge", f"lumen_kv_cache_usage_ratio {live['kv_usage']:.4f}",
            "# TYPE lumen_running_requests gauge", f"lumen_running_requests {live['running']}",
            "# TYPE lumen_waiting_requests gauge", f"lumen_waiting_requests {live['waiting']}",
            "# TYPE lumen_preemptions_total counter",
            f"lumen_preemptions_total {live['preemptions']}",
            "# TYPE lumen_prefix_cache_hit_ratio gauge",
            f"lumen_prefix_cache_hit_ratio {live.get('prefix_hit_rate', 0.0):.4f}",
        ]
        return PlainTextResponse("\n".join(lines) + "\n")

    async def _deltas(prompt, params, rid, lora, stop):
        """One engine stream through the detokenizer and the stop-string check: yields
        (text delta, finish_reason | None, seq) per engine step that produced tokens."""
        detok = IncrementalDetokenizer(tok)
        last = None
        try:
            async for seq in aengine.stream(prompt, params, rid, lora):
                last = seq
                fin = seq.finish_reason if seq.finished else None
                d = detok.step(seq.output_ids)
                if fin:
                    d += detok.flush(seq.output_ids)
                out = stop.feed(d, final=fin is not None)
                if stop.stopped:
                    fin = "stop"
                yield out, fin, seq
                if fin is not None:
                    break   # a stop string ends the stream early: the engine request is aborted
        finally:
            if last is not None:
                stats.observe(last)

    async def _one(prompt, params, rid, lora, stops, include_stop, on_delta=None):
        """Drive one engine stream to completion.  Calls ``on_delta(text, finish_reason, seq)``
        per engine step (streaming); returns (text, seq, finish_reason)."""
        stop = StopChecker(stops, include_stop)
        last, fin = None, None
        async for out, fin, seq in _deltas(prompt, params, rid, lora, stop):
            last = seq
            if on_delta is not None:
                await on_delta(out, fin, seq)
        return stop.text, last, fin

    async def _run(prompt, params, chat: bool, stream: bool, model: str, body: Dict[str, Any]):
        rid = ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex
        lora = model if model in loras else None  # OpenAI "model" selects a served adapter
        created = int(time.time())
        stats.requests += 1
        obj = "chat.completion" if chat else "text_completion"
        echo = not chat and bool(body.get("echo", False))
        score_only = echo and body.get("max_tokens") == 0   # score the prompt, generate nothing
        try:
            stops = _stops(body)
            n, best_of = _n_best_of(body, stream)
            want_lp = _logprob_request(body, chat, params)
            if score_only and stream:
                raise ValueError("echo with max_tokens 0 is not streamed")
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        if score_only:
            params.max_tokens = 1   # one token is sampled (and dropped): the prompt forward
        include_stop = bool(body.get("include_stop_str_in_output", False))
        prompt_text = (prompt if isinstance(prompt, str) else decode(list(prompt))) if echo else ""

        def tops_of(seq, a=0):
            t = getattr(seq, "output_top_logprobs", None) or []
            n_out = len(seq.output_ids)
            return t[a:n_out] if len(t) >= n_out else [None] * (n_out - a)

        def lp_object(seq, a, with_prompt, end=None):
            """logprobs of output tokens a..end (and, for echo, of the prompt first)."""
            ids, lps, tops = (seq.output_ids[a:end], seq.output_logprobs[a:end],
                              tops_of(seq, a)[:None if end is None else end - a])
            if chat:
                return chat_logprobs(decode, ids, lps, tops)
            if with_prompt:
                ps = list(getattr(seq, "prompt_scores", None) or [])
                ps += [None] * (len(seq.prompt_ids) - len(ps))
                ids = list(seq.prompt_ids) + list(ids)
                lps = [None if x is None else x[0] for x in ps] + list(lps)
                tops = [None if x is None else x[1] for x in ps] + list(tops)
            return completion_logprobs(decode, ids, lps, tops)

        def sub_params(i):
            p = SamplingParams(**vars(params))
            if p.seed is not None:
                p.seed = p.seed + i     # distinct choices under a fixed seed
            return p

        head = sse_head(rid, chat, created, model)

        def sse(delta_text, finish, index=0, lpo=None):
            if lpo is None:
                return sse_event(head, chat, delta_text, finish, index)
            return "data: %s\n\n" % json.dumps(stream_chunk(rid, chat, created, model, delta_text,
                                                            finish, index, lpo))

        def streamed(out, fin, seq, index, st):
            """One event; ``st`` = [tokens already reported, first event pending]."""
            lpo = None
            first = st[1]
            st[1] = False
            if first and echo:
                out = prompt_text + out
            if want_lp:
                lpo = lp_object(seq, st[0], first and echo)
                st[0] = len(seq.output_ids)
            return sse(out, fin, index, lpo)

        if stream and n == 1:
            async def gen1():
                # one choice: the engine stream drives the response directly (no per-token
                # queue hop or task switch)
                if chat:
                    first = {"id": rid, "object": "chat.completion.chunk", "created": created,
                             "model": model, "choices": [{"index": 0,
                                                          "delta": {"role": "assistant"},
                                                          "finish_reason": None}]}
                    yield f"data: {json.dumps(first)}\n\n"
                stop = StopChecker(stops, include_stop)
                st = [0, True]
                try:
                    async for out, fin, seq in _deltas(prompt, sub_params(0), rid, lora, stop):
                        yield (streamed(out, fin, seq, 0, st) if want_lp or echo
                               else sse(out, fin))
                except ValueError as e:
                    stats.errors += 1
                    yield f"data: {json.dumps({'error': {'message': str(e)}})}\n\n"
                yield "data: [DONE]\n\n"
            return StreamingResponse(gen1(), media_type="text/event-stream")

        if stream:
            async def gen():
                q: asyncio.Queue = asyncio.Queue()

                async def run_choice(i):
                    st = [0, True]

                    async def on_delta(text, fin, seq):
                        # one event per engine step that produced tokens, even when the text
                        # delta is still empty (incomplete UTF-8 / held-back stop prefix):
                        # clients see token timing (TTFT, inter-token latency)
                        await q.put(streamed(text, fin, seq, i, st))
                    try:
                        await _one(prompt, sub_params(i), f"{rid}-{i}" if n > 1 else rid, lora,
                                   stops, include_stop, on_delta)
                    except ValueError as e:
                        stats.errors += 1
                        await q.put(f"data: {json.dumps({'error': {'message': str(e)}})}\n\n")
                    finally:
                        await q.put(None)

                if chat:
                    for i in range(n):
                        first = {"id": rid, "object": "chat.completion.chunk",
                                 "created": created, "model": model,
                                 "choices": [{"index": i, "delta": {"role": "assistant"},
                                              "finish_reason": None}]}
                        yield f"data: {json.dumps(first)}\n\n"
                tasks = [asyncio.ensure_future(run_choice(i)) for i in range(n)]
                live = n
                try:
                    while live:
                        item = await q.get()
                        if item is None:
                            live -= 1
                            continue
                        yield item
                finally:
                    for t in tasks:
                        if not t.done():
                            t.cancel()
                yield "data: [DONE]\n\n"
            return StreamingResponse(gen(), media_type="text/event-stream")

        try:
            res = await asyncio.gather(*[
                _one(prompt, sub_params(i), f"{rid}-{i}" if best_of > 1 else rid, lora, stops,
                     include_stop) for i in range(best_of)])
        except ValueError as e:
            stats.errors += 1
            raise HTTPException(status_code=400, detail=str(e))
        if best_of > n:  # OpenAI best_of: the n choices with the highest total log probability
            res = sorted(res, key=lambda r: -sum(r[1].output_logprobs))[:n]
        choices = []
        n_out = 0
        for i, (text, seq, fin) in enumerate(res):
            n_gen = len(seq.output_ids)
            if score_only:   # the sampled token is not part of the answer
                text, fin, n_gen = "", "length", 0
            n_out += n_gen
            lp = lp_object(seq, 0, echo, n_gen) if want_lp else None
            if chat:
                choices.append({"index": i, "message": {"role": "assistant", "content": text},
                                "logprobs": lp, "finish_reason": fin})
            else:
                choices.append({"index": i, "text": prompt_text + text, "logprobs": lp,
                                "finish_reason": fin})
        p_tok = len(res[0][1].prompt_ids)
        usage = {"prompt_tokens": p_tok, "completion_tokens": n_out,
                 "total_tokens": p_tok + n_out}
        return JSONResponse({"id": rid, "object": obj, "created": created, "model": model,
                             "choices": choices, "usage": usage})

    @app.post("/v1/completions")
    async def completions(req: Request):
        body = await req.json()
        prompt: Union[str, List[int], List[str]] = body.get("prompt", "")
        if isinstance(prompt, list) and prompt and isinstance(prompt[0], str):
            if len(prompt) != 1:
                raise HTTPException(status_code=400, detail="batched string prompts: send one per request")
            prompt = prompt[0]
        try:
            params = _params(body, aengine.eos_id)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        return await _run(prompt, params, False, bool(body.get("stream", False)),
                          body.get("model", name), body)

    @app.post("/v1/chat/completions")
    async def chat(req: Request):
        body = await req.json()
        msgs = body.get("messages") or []
        if not msgs:
            raise HTTPException(status_code=400, detail="messages required")
        try:
            params = _params(body, aengine.eos_id)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e))
        return await _run(llama2_chat_prompt(msgs), params, True, bool(body.get("stream", False)),
                          body.get("model", name), body)

    app.state.stats = stats
    return app
