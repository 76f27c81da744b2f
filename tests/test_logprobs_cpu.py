"""OpenAI logprobs parity on CPU: top alternatives per generated token, prompt scoring
(``echo`` + ``logprobs``, ``max_tokens: 0``), chat ``logprobs`` / ``top_logprobs``, streamed
logprobs; engine values against the model's own log-softmax; the engine-core / API process
protocol carries them."""
import json
import queue
import threading

import pytest
import torch

from lumen.models import build_model
from lumen.serve.engine import AsyncEngine, EngineConfig, LLMEngine
from lumen.serve.sequence import SamplingParams


@pytest.fixture(scope="module")
def model():
    torch.manual_seed(0)
    m = build_model("tiny-llama-gqa", dtype=torch.float32, device="cpu", init="random", seed=1)
    with torch.no_grad():
        for p in m.parameters():
            if p.dim() == 2:
                p.mul_(5.0)
    m.eval()
    return m


def _engine(model, **kw):
    cfg = EngineConfig(model="tiny-llama-gqa", device="cpu", max_model_len=256, block_size=4,
                       use_graphs=False, num_blocks=128, **kw)
    return LLMEngine(cfg, model=model)


def _ref_logprobs(model, ids):
    with torch.no_grad():
        return torch.log_softmax(model(torch.tensor([ids])).view(len(ids), -1).float(), -1)


@pytest.mark.parametrize("async_sched", [True, False])
def test_engine_prompt_scores_and_alternatives(model, async_sched):
    # an 8-token budget splits the 17-token prompt over three chunks: scores accumulate
    eng = _engine(model, max_num_batched_tokens=8, async_scheduling=async_sched)
    prompt = list(range(3, 20))
    plain = eng.add_request([7, 8, 9], SamplingParams(max_tokens=6, temperature=0.0,
                                                      ignore_eos=True))
    s = eng.add_request(prompt, SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True,
                                               top_logprobs=3, prompt_logprobs=2))
    while eng.has_work:
        eng.step()
    assert plain.finished and not plain.output_top_logprobs and not plain.prompt_scores
    lp = _ref_logprobs(model, prompt + s.output_ids)
    assert len(s.prompt_scores) == len(prompt) and s.prompt_scores[0] is None
    for j in range(1, len(prompt)):
        score, alts = s.prompt_scores[j]
        assert abs(score - lp[j - 1, prompt[j]].item()) < 1e-4
        assert [a for a, _ in alts] == lp[j - 1].topk(2).indices.tolist()
    assert len(s.output_top_logprobs) == len(s.output_ids) == 5
    for i, t in enumerate(s.output_ids):
        row = lp[len(prompt) - 1 + i]
        top = row.topk(3)
        assert [a for a, _ in s.output_top_logprobs[i]] == top.indices.tolist()
        assert abs(s.output_top_logprobs[i][0][1] - top.values[0].item()) < 1e-4
        assert abs(s.output_logprobs[i] - row[t].item()) < 1e-4
    assert eng.blocks.num_free == eng.blocks.num_blocks


def _check_api(c, model, tok):
    base = {"prompt": [5, 6, 7, 8, 9, 10], "max_tokens": 6, "temperature": 0,
            "ignore_eos": True}
    j = c.post("/v1/completions", json=dict(base, logprobs=3)).json()["choices"][0]
    lpo = j["logprobs"]
    assert len(lpo["tokens"]) == len(lpo["token_logprobs"]) == len(lpo["top_logprobs"]) == 6
    assert all(1 <= len(d) <= 4 for d in lpo["top_logprobs"])
    assert lpo["text_offset"] == sorted(lpo["text_offset"]) and lpo["text_offset"][0] == 0
    for lp_, d in zip(lpo["token_logprobs"], lpo["top_logprobs"]):
        assert abs(max(d.values()) - lp_) < 1e-5   # greedy: the chosen token is the top one
    # echo + max_tokens 0: score the prompt, generate nothing (lm-eval loglikelihood)
    e = c.post("/v1/completions", json=dict(base, max_tokens=0, echo=True, logprobs=1)).json()
    ch = e["choices"][0]
    ids = base["prompt"]
    assert ch["text"] == tok.decode(ids) and e["usage"]["completion_tokens"] == 0
    lps = ch["logprobs"]["token_logprobs"]
    assert len(lps) == len(ids) and lps[0] is None and ch["logprobs"]["top_logprobs"][0] is None
    ref = _ref_logprobs(model, ids)
    for k in range(1, len(ids)):
        assert abs(lps[k] - ref[k - 1, ids[k]].item()) < 1e-4
    # echo with generation: prompt then completion, one logprobs object over both
    e2 = c.post("/v1/completions", json=dict(base, echo=True, logprobs=0)).json()["choices"][0]
    assert e2["text"].startswith(tok.decode(ids))
    assert len(e2["logprobs"]["tokens"]) == len(ids) + 6
    # chat
    cj = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hi"}],
                                               "max_tokens": 4, "temperature": 0,
                                               "logprobs": True, "top_logprobs": 2}).json()
    content = cj["choices"][0]["logprobs"]["content"]
    assert len(content) == 4 and all(len(x["top_logprobs"]) == 2 for x in content)
    assert all(x["bytes"] == list(x["token"].encode()) for x in content)
    # streamed logprobs == non-streamed
    with c.stream("POST", "/v1/completions", json=dict(base, logprobs=3, stream=True)) as s:
        lines = [ln for ln in s.iter_lines() if ln]
    chunks = [json.loads(ln[6:]) for ln in lines[:-1]]
    toks = [t for ch in chunks for t in (ch["choices"][0]["logprobs"] or {}).get("tokens", [])]
    assert toks == lpo["tokens"]
    assert c.post("/v1/completions", json=dict(base, logprobs=21)).status_code == 400


def test_openai_logprobs_in_process(model):
    from starlette.testclient import TestClient

    from lumen.serve.api_server import create_app

    eng = _engine(model)
    ae = AsyncEngine(eng)
    try:
        _check_api(TestClient(create_app(ae, "tiny")), model, eng.tokenizer)
    finally:
        ae.shutdown()
    assert eng.blocks.num_free == eng.blocks.num_blocks


def test_openai_logprobs_through_engine_core(model):
    """The same checks with the engine core behind the process protocol (queues)."""
    from starlette.testclient import TestClient

    from lumen.serve.api_server import create_app
    from lumen.serve.frontend import EngineCoreClient, run_engine_core

    eng = _engine(model)
    req_q, out_q = queue.Queue(), queue.Queue()
    core = threading.Thread(target=run_engine_core, args=(eng, req_q, [out_q]), daemon=True)
    core.start()
    client = EngineCoreClient(req_q, out_q, eng.tokenizer, "tiny", 256, eng.eos_id)
    try:
        _check_api(TestClient(create_app(client, "tiny")), model, eng.tokenizer)
    finally:
        req_q.put(("stop",))
        core.join(timeout=30)
        out_q.put(None)


def test_tokenize_detokenize_version_endpoints(model):
    from starlette.testclient import TestClient

    from lumen.serve.api_server import create_app

    eng = _engine(model)
    ae = AsyncEngine(eng)
    try:
        c = TestClient(create_app(ae, "tiny"))
        t = c.post("/tokenize", json={"prompt": "hello world"}).json()
        assert t["count"] == len(t["tokens"]) > 0 and t["max_model_len"] == 256
        assert c.post("/detokenize", json={"tokens": t["tokens"]}).json()["prompt"] == "hello world"
        m = c.post("/tokenize", json={"messages": [{"role": "user", "content": "hi"}]}).json()
        assert m["count"] > t["count"] - 5
        assert c.post("/detokenize", json={"tokens": "x"}).status_code == 400
        assert "version" in c.get("/version").json()
    finally:
        ae.shutdown()
