"""Speculative decoding by prompt lookup (vLLM ``--speculative-model "[ngram]"``): drafts are
verified in one forward and greedy outputs stay identical to one-token decoding -- with oracle
drafts (all / part / none accepted), with the real n-gram proposer, next to sampled and
penalised sequences, and with stop tokens inside an accepted draft."""
import pytest
import torch

from lumen.models import build_model
from lumen.serve.engine import EngineConfig, LLMEngine
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


def naive_greedy(model, ids, n):
    ids, out = list(ids), []
    with torch.no_grad():
        for _ in range(n):
            t = int(model(torch.tensor([ids])).view(len(ids), -1)[-1].argmax())
            out.append(t)
            ids.append(t)
    return out


def _engine(model, k=4, **kw):
    cfg = EngineConfig(model="tiny-llama-gqa", device="cpu", max_model_len=256, block_size=4,
                       use_graphs=False, num_blocks=256, num_speculative_tokens=k, **kw)
    return LLMEngine(cfg, model=model)


GREEDY = dict(temperature=0.0, ignore_eos=True)
PROMPTS = [[5, 9, 33, 7] * 4, list(range(3, 20)), [42, 43, 44]]


def test_lookup_finds_latest_longest_match(model):
    eng = _engine(model)
    ids = [1, 2, 3, 9, 9, 1, 2, 3, 4, 5, 6, 7, 1, 2, 3]
    assert eng._lookup(ids, 3) == [4, 5, 6]      # latest occurrence of [1, 2, 3]
    assert eng._lookup([8, 1, 2, 7, 5, 2], 2) == [7, 5]   # falls back to a 1-gram
    assert eng._lookup([1, 2, 3], 4) == []
    # the incremental index of a growing sequence gives the same answers as a fresh one
    from lumen.serve.sequence import Sequence
    seq = Sequence([1, 2, 3], SamplingParams())
    grow = [1, 2, 3]
    for t in [9, 9, 1, 2, 3, 4, 5, 6, 7, 1, 2, 3]:
        grow.append(t)
        assert eng._lookup(grow, 3, seq) == eng._lookup(grow, 3)


def test_oracle_drafts_all_part_none_accepted(model):
    refs = [naive_greedy(model, p, 24) for p in PROMPTS]
    eng = _engine(model, k=5)

    def oracle(ids, k):
        for p, r in zip(PROMPTS, refs):
            full = p + r
            if ids == full[:len(ids)]:
                d = full[len(ids):len(ids) + k]
                if p is PROMPTS[1] and len(d) > 2:
                    d[2] = (d[2] + 1) % 500       # this prompt's drafts fail at their 3rd token
                return [] if p is PROMPTS[2] else d
        raise AssertionError("unexpected sequence")

    eng._lookup = lambda ids, k, s=None: oracle(ids, k)
    seqs = eng.generate(PROMPTS, SamplingParams(max_tokens=24, **GREEDY))
    for s, r in zip(seqs, refs):
        assert s.output_ids == r
        assert len(s.output_logprobs) == 24
    st = eng.stats
    assert st["spec_accepted"] > 0 and st["spec_accepted"] < st["spec_proposed"]
    assert eng.blocks.num_free == eng.blocks.num_blocks
    # alone, the always-right drafts give k + 1 tokens per step: 1 prefill + 4 verify steps
    solo = _engine(model, k=5)
    solo._lookup = lambda ids, k, s=None: oracle(ids, k)
    s = solo.generate([PROMPTS[0]], SamplingParams(max_tokens=24, **GREEDY))[0]
    assert s.output_ids == refs[0] and solo.stats["steps"] == 5


def test_prompt_lookup_next_to_sampled_and_penalised(model):
    prompts = [[5, 9, 33, 7] * 4, list(range(3, 20)) * 2, [7, 7, 7, 7, 7, 7]]
    seqs = _engine(model).generate(prompts, SamplingParams(max_tokens=40, **GREEDY))
    for p, s in zip(prompts, seqs):
        assert s.output_ids == naive_greedy(model, p, 40)
    # a sampled (top_k=1: deterministic) and a penalised request ride as plain decode rows
    mixed = [SamplingParams(max_tokens=20, **GREEDY),
             SamplingParams(max_tokens=20, temperature=0.7, top_k=1, ignore_eos=True),
             SamplingParams(max_tokens=20, frequency_penalty=1.0, **GREEDY)]
    pr = [[5, 9, 33, 7] * 4, [11, 12, 13], [20, 21, 22, 20, 21]]

    def run(k):
        eng = _engine(model, k=k)
        ss = [eng.add_request(p, sp) for p, sp in zip(pr, mixed)]
        while eng.has_work:
            eng.step()
        return [s.output_ids for s in ss]

    assert run(4) == run(0)


def test_stop_token_inside_accepted_draft(model):
    p = PROMPTS[0]
    ref = naive_greedy(model, p, 16)
    eng = _engine(model, k=6)
    eng._lookup = lambda ids, k, s=None: (p + ref)[len(ids):len(ids) + k]
    s = eng.generate([p], SamplingParams(max_tokens=16, temperature=0.0,
                                          stop_token_ids=[ref[5]], ignore_eos=True))[0]
    stop_at = ref.index(ref[5])
    assert s.output_ids == ref[:stop_at + 1] and s.finish_reason == "stop"
    s2 = eng.generate([p], SamplingParams(max_tokens=7, **GREEDY))[0]
    assert s2.output_ids == ref[:7] and s2.finish_reason == "length"
    assert eng.blocks.num_free == eng.blocks.num_blocks


def test_lookup_index_is_windowed_and_bounded():
    """the per-sequence n-gram index is bounded by ngram_window (pruned as it
    slides) and still finds a repeat inside the window."""
    from types import SimpleNamespace

    from lumen.serve.engine import EngineConfig, LLMEngine

    eng = SimpleNamespace(cfg=EngineConfig(ngram_window=64, ngram_max=4, ngram_min=1),
                          _ngram_key=LLMEngine._ngram_key)
    s = SimpleNamespace(ngram_idx={}, ngram_upto=0)
    ids = list(range(1000, 1600))                       # 600 distinct tokens
    for L in range(2, len(ids) + 1, 7):
        LLMEngine._lookup(eng, ids[:L], 3, s)
    LLMEngine._lookup(eng, ids, 3, s)
    assert len(s.ngram_idx) <= 64 * 4 + 8
    # a repeat of a recent n-gram is proposed, one from before the window is not
    rec = ids + ids[-10:-8]
    assert LLMEngine._lookup(eng, rec, 3, s) == ids[-8:-5]
    s2 = SimpleNamespace(ngram_idx={}, ngram_upto=0)
    old = ids + ids[5:7]
    assert LLMEngine._lookup(eng, old, 3, s2) == []
