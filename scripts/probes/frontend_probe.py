"""The OpenAI HTTP front-end under serving load, without a GPU: a fake engine core emits one
token for every live request each ``--step-ms`` (the decode-step cadence of the real engine at
256 streams), the real API process (lumen.serve.frontend.api_process_main) streams them, the real
load client (lumen.bench.async_client) measures.  Whatever ITL the client sees above the step
period is front-end (API process + client) overhead.

    python scripts/probes/frontend_probe.py [--requests 256] [--step-ms 20] [--max-tokens 128]
"""
import argparse
import json
import multiprocessing as mp
import os
import queue
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)


def fake_core(req_q, out_qs, step_s, prefill_s):
    """Admit requests; a request's first token comes one prefill step after arrival, then one
    token per decode step for all live requests."""
    live = {}
    stop = False
    next_t = time.perf_counter()
    while not stop:
        while True:
            try:
                op = req_q.get_nowait() if live else req_q.get(timeout=0.05)
            except queue.Empty:
                break
            if op[0] == "add":
                _, rid, ids, pdict, arrival, lora = op[:6]
                live[rid] = [pdict["max_tokens"], 0, time.perf_counter() + prefill_s,
                             op[6] if len(op) > 6 else 0]
            elif op[0] == "abort":
                live.pop(op[1], None)
            elif op[0] == "stop":
                stop = True
        if not live:
            next_t = time.perf_counter()
            continue
        now = time.perf_counter()
        if now < next_t:
            time.sleep(next_t - now)
        next_t += step_s
        now = time.perf_counter()
        updates = {}
        for rid, st in list(live.items()):
            if now < st[2]:
                continue
            st[1] += 1
            fin = "length" if st[1] >= st[0] else None
            # no text (byte tokenizer), as in the bench
            updates.setdefault(st[3], []).append((rid, [1000 + st[1]], [], fin))
            if fin:
                del live[rid]
        for o, ups in updates.items():
            out_qs[o].put(("step", ups, {"kv_usage": 0.0, "running": len(live), "waiting": 0,
                                         "preemptions": 0}))


def api_profiled(path, *args):
    """api_process_main under cProfile; SIGTERM dumps the stats to ``path``."""
    import cProfile
    import signal

    from lumen.serve.frontend import api_process_main

    prof = cProfile.Profile()

    def dump(*_):
        prof.disable()
        prof.dump_stats(path)
        os._exit(0)

    signal.signal(signal.SIGTERM, dump)
    prof.enable()
    api_process_main(*args)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--step-ms", type=float, default=20.0)
    ap.add_argument("--prefill-ms", type=float, default=50.0)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--profile", default=None, help="cProfile the API process into this file")
    ap.add_argument("--profile-client", default=None, help="cProfile the load client into this file")
    ap.add_argument("--procs", type=int, default=1, help="load-client processes")
    ap.add_argument("--api", type=int, default=1, help="API server processes")
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    if a.profile:
        req_q, out_qs = ctx.Queue(), [ctx.Queue()]
        args = (req_q, out_qs[0], "llama2-7b", 1024, "127.0.0.1", port, "lumen", 32000)
        apis = [ctx.Process(target=api_profiled, args=(a.profile,) + args, daemon=True)]
        apis[0].start()
    else:
        from lumen.serve.frontend import start_api_servers

        req_q, out_qs, apis = start_api_servers(a.api, "llama2-7b", 1024, "127.0.0.1", port,
                                                "lumen", 32000)
    core = ctx.Process(target=fake_core, args=(req_q, out_qs, a.step_ms / 1000, a.prefill_ms / 1000),
                       daemon=True)
    core.start()
    url = f"http://127.0.0.1:{port}"
    t0 = time.time()
    while True:
        try:
            urllib.request.urlopen(url + "/health", timeout=2)
            break
        except Exception:
            assert time.time() - t0 < 60
            time.sleep(0.2)
    prof = ["-m", "cProfile", "-o", a.profile_client] if a.profile_client else []
    out = subprocess.run([sys.executable] + prof + ["-m", "lumen.bench.async_client", "--url", url,
                          "--num-requests", str(a.requests), "--concurrency", str(a.requests),
                          "--prompt-len", "512", "--max-tokens", str(a.max_tokens), "--warmup", "16",
                          "--procs", str(a.procs)],
                         capture_output=True, cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT))
    req_q.put(("stop",))
    for p in apis:
        p.terminate()
    for p in apis:
        p.join(10)
    line = [l for l in out.stdout.decode().splitlines() if l.startswith("{")]
    print(line[-1] if line else out.stderr.decode()[-2000:])


if __name__ == "__main__":
    main()
