"""Engine core / API front-end split across processes.

The GPU process (rank 0 of the TP group) runs the scheduler + model loop (``run_engine_core``);
the OpenAI HTTP server runs in a spawned child process that never touches the GPU and talks to
the core through two multiprocessing queues.  With both in one process (``AsyncEngine``: engine
thread + asyncio loop) every streamed token's JSON/SSE work competes with the engine's Python
bookkeeping for the GIL; at 256 concurrent streams that serialisation, not the GPU, set the
client-side inter-token latency (1.2 s vs 22 ms engine-side).  The split keeps the engine step
loop free of HTTP work, as vLLM's engine-core process does.

Several API processes (``--api-server-count``, as in later vLLM releases) may share one
engine core: each listens on the same port (SO_REUSEPORT: the kernel spreads the connections),
all of them put requests on the one request queue, and each has its own output queue -- the core
routes every request's tokens to the front-end that submitted it (each process's ``/metrics``
counts the requests it served; the engine-state gauges are the core's).  At 256 concurrent streams one
Python front-end is CPU-bound (request intake + ~13k SSE events/s), and its lag reads as
inter-token latency at the client.

Protocol (all plain tuples/lists, pickled by multiprocessing):
  front -> core: ("add", rid, prompt_ids, params_dict, arrival, lora_name|None, front_index)
                 | ("abort", rid) | ("stop",)
  core -> front: ("step", [(rid, new_ids, new_logprobs, finish_reason|None[, extras]), ...],
                  stats)   extras (only for requests asking logprob alternatives / prompt
                  scores): {"top": new tokens' alternatives, "prompt": prompt scores (once)}
                 ("error", rid, message)
"""
from __future__ import annotations

import asyncio
import dataclasses
import queue
import threading
import time
import uuid
from typing import Dict, List, Optional

from .sequence import SamplingParams


# ------------------------------------------------------------------------------------------
# GPU process side
# ------------------------------------------------------------------------------------------

def run_engine_core(engine, req_q, out_q, idle_sleep: float = 0.0005) -> None:
    """Serve requests from ``req_q`` until a ("stop",) message; one out message per step and
    front-end.  ``out_q``: one queue, or a list (one per API process, indexed by the "add"
    message's front index)."""
    outs = list(out_q) if isinstance(out_q, (list, tuple)) else [out_q]
    live: Dict[str, object] = {}
    sent: Dict[str, int] = {}
    origin: Dict[str, int] = {}
    stop = False
    while not stop:
        block = not engine.has_work
        while True:
            try:
                op = req_q.get(timeout=0.05) if block else req_q.get_nowait()
            except queue.Empty:
                break
            block = False
            kind = op[0]
            if kind == "add":
                _, rid, ids, pdict, arrival, lora = op[:6]
                o = op[6] if len(op) > 6 and 0 <= op[6] < len(outs) else 0
                try:
                    seq = engine.add_request(ids, SamplingParams(**pdict), rid, lora)
                    seq.arrival = arrival
                    live[rid] = seq
                    sent[rid] = 0
                    origin[rid] = o
                except Exception as e:  # noqa: BLE001 - report to the request's stream
                    outs[o].put(("error", rid, str(e)))
            elif kind == "abort":
                engine.abort(op[1])
                live.pop(op[1], None)
                sent.pop(op[1], None)
                origin.pop(op[1], None)
            elif kind == "stop":
                stop = True
        if stop or not engine.has_work:
            if not engine.has_work:
                time.sleep(idle_sleep)
            continue
        try:
            seqs = engine.step()
        except Exception as e:  # noqa: BLE001 - surface to every open stream, then fail
            for rid in list(live):
                outs[origin.get(rid, 0)].put(("error", rid, repr(e)))
            raise
        updates: Dict[int, list] = {}
        for s in seqs:
            rid = s.request_id
            if rid not in live:
                continue
            k = sent[rid]
            new = s.output_ids[k:]
            lps = s.output_logprobs[k:] if s.output_logprobs else []
            sent[rid] = len(s.output_ids)
            fin = s.finish_reason if s.finished else None
            if s.params.wants_extras:
                ex = {"top": s.output_top_logprobs[k:]}
                if k == 0 and s.prompt_scores:
                    ex["prompt"] = s.prompt_scores
                updates.setdefault(origin[rid], []).append((rid, new, lps, fin, ex))
            else:
                updates.setdefault(origin[rid], []).append((rid, new, lps, fin))
            if fin is not None:
                live.pop(rid, None)
                sent.pop(rid, None)
                origin.pop(rid, None)
        if updates:
            sch = engine.scheduler
            stats = {"kv_usage": engine.blocks.usage(), "running": len(sch.running),
                     "waiting": len(sch.waiting), "preemptions": sch.num_preemptions,
                     "prefix_hit_rate": engine.blocks.hit_rate}
            for o, ups in updates.items():
                outs[o].put(("step", ups, stats))


# ------------------------------------------------------------------------------------------
# API process side
# ------------------------------------------------------------------------------------------

@dataclasses.dataclass
class SeqView:
    """Client-side mirror of a Sequence (same attribute names the API code reads)."""
    prompt_ids: List[int]
    request_id: str
    arrival: float
    output_ids: List[int] = dataclasses.field(default_factory=list)
    output_logprobs: List[float] = dataclasses.field(default_factory=list)
    token_times: List[float] = dataclasses.field(default_factory=list)
    first_token_time: Optional[float] = None
    finish_reason: Optional[str] = None
    output_top_logprobs: List[list] = dataclasses.field(default_factory=list)
    prompt_scores: List[object] = dataclasses.field(default_factory=list)

    @property
    def finished(self) -> bool:
        return self.finish_reason is not None

    @property
    def length(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)


class EngineCoreClient:
    """The ``AsyncEngine`` interface (``stream``, ``tokenizer``, ``live_stats`` ...) backed by an
    engine core in another process."""

    def __init__(self, req_q, out_q, tokenizer, model_name: str, max_model_len: int,
                 eos_id: Optional[int], lora_names: Optional[List[str]] = None, index: int = 0):
        self.req_q, self.out_q = req_q, out_q
        self.index = index  # which of the core's output queues carries this front-end's tokens
        self.lora_names = list(lora_names or [])
        self.tokenizer = tokenizer
        self.model_name = model_name
        self.max_model_len = max_model_len
        self.eos_id = eos_id
        self._streams: Dict[str, tuple] = {}
        self._stats = {"kv_usage": 0.0, "running": 0, "waiting": 0, "preemptions": 0}
        self._reader = threading.Thread(target=self._read, name="lumen-core-reader", daemon=True)
        self._reader.start()

    def live_stats(self) -> dict:
        return dict(self._stats)

    def _read(self):
        while True:
            msg = self.out_q.get()
            if msg is None:
                return
            if msg[0] == "step":
                _, updates, stats = msg
                self._stats = stats
                now = time.perf_counter()
                by_loop: Dict[object, list] = {}
                for u in updates:
                    st = self._streams.get(u[0])
                    if st is None:
                        continue
                    by_loop.setdefault(st[0], []).append(
                        (st[1], ("token", (u[1], u[2], u[3], now, u[4] if len(u) > 4 else None))))
                for loop, items in by_loop.items():
                    loop.call_soon_threadsafe(_deliver, items)
            elif msg[0] == "error":
                st = self._streams.get(msg[1])
                if st is not None:
                    st[0].call_soon_threadsafe(_deliver, [(st[1], ("error", msg[2]))])

    async def stream(self, prompt, params: SamplingParams, request_id: Optional[str] = None,
                     lora: Optional[str] = None):
        rid = request_id or uuid.uuid4().hex
        ids = self.tokenizer.encode(prompt) if isinstance(prompt, str) else list(prompt)
        if not ids:
            raise ValueError("empty prompt")
        if len(ids) >= self.max_model_len:
            raise ValueError(f"prompt ({len(ids)} tokens) does not fit max_model_len "
                             f"{self.max_model_len}")
        q: asyncio.Queue = asyncio.Queue()
        self._streams[rid] = (asyncio.get_running_loop(), q)
        view = SeqView(ids, rid, time.perf_counter())
        self.req_q.put(("add", rid, ids, dataclasses.asdict(params), view.arrival, lora,
                        self.index))
        try:
            while True:
                kind, payload = await q.get()
                if kind == "error":
                    raise ValueError(payload)
                new, lps, fin, now, ex = payload
                if new and view.first_token_time is None:
                    view.first_token_time = now
                view.output_ids.extend(new)
                view.output_logprobs.extend(lps)
                if ex is not None:
                    view.output_top_logprobs.extend(ex.get("top", []))
                    if "prompt" in ex:
                        view.prompt_scores = list(ex["prompt"])
                view.token_times.extend([now] * len(new))
                view.finish_reason = fin
                yield view
                if fin is not None:
                    break
        finally:
            self._streams.pop(rid, None)
            if not view.finished:
                self.req_q.put(("abort", rid))  # client went away: free its KV blocks

    def shutdown(self):
        self.req_q.put(("stop",))


def _deliver(items):
    for q, item in items:
        q.put_nowait(item)


def api_process_main(req_q, out_q, model: str, max_model_len: int, host: str, port: int,
                     served_model_name: Optional[str], vocab_size: int,
                     lora_names: Optional[List[str]] = None, index: int = 0,
                     reuse_port: bool = False) -> None:
    """Entry point of a spawned HTTP process (no GPU).  ``reuse_port``: one of several API
    processes listening on the same port (SO_REUSEPORT)."""
    import os

    import uvicorn

    parent = os.getppid()

    def _watch():  # never outlive the engine process (e.g. after a SIGKILL)
        while os.getppid() == parent:
            time.sleep(1.0)
        os._exit(0)

    threading.Thread(target=_watch, daemon=True).start()

    from ..data.tokenizer import load_tokenizer
    from .api_server import create_app

    tok = load_tokenizer(model, vocab_size)
    eos = getattr(tok, "eos_token_id", None)
    client = EngineCoreClient(req_q, out_q, tok, served_model_name or model, max_model_len, eos,
                              lora_names, index)
    app = create_app(client, served_model_name)
    if not reuse_port:
        uvicorn.run(app, host=host, port=port, log_level="warning")
        return
    import socket

    sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    sock.bind((host, port))
    sock.listen(2048)
    uvicorn.Server(uvicorn.Config(app, log_level="warning")).run(sockets=[sock])


def start_api_servers(count: int, model: str, max_model_len: int, host: str, port: int,
                      served_model_name: Optional[str], vocab_size: int,
                      lora_names: Optional[List[str]] = None):
    """Spawn ``count`` API processes on ``host:port`` sharing one request queue; returns
    (request queue, [output queue per process], [processes]) for ``run_engine_core``."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    req_q = ctx.Queue()
    out_qs, procs = [], []
    for i in range(max(1, count)):
        out_q = ctx.Queue()
        p = ctx.Process(target=api_process_main, name=f"lumen-api{i}",
                        args=(req_q, out_q, model, max_model_len, host, port, served_model_name,
                              vocab_size, lora_names, i, count > 1), daemon=True)
        p.start()
        out_qs.append(out_q)
        procs.append(p)
    return req_q, out_qs, procs
