"""Serving on the GPU: HIP paged decode + graphs reproduce full-recompute logits."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_engine_decode_matches_full_forward():
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.model_runner import StepInput
    from lumen.serve.sequence import SamplingParams

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
    m.eval()
    for graphs in (False, True):
        eng = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=512,
                                     block_size=16, num_blocks=128, use_graphs=graphs), model=m)
        prompts = [[5, 9, 33, 7] * 10, list(range(3, 60)), [42, 43]]
        seqs = [eng.add_request(p, SamplingParams(max_tokens=20, temperature=0.0, ignore_eos=True))
                for p in prompts]
        while eng.has_work:
            eng.step()
        for p, s in zip(prompts, seqs):
            ids = torch.tensor([p + s.output_ids[:-1]], device=dev)
            with torch.no_grad():
                full = m(ids).float().view(ids.shape[1], -1)
            # teacher-forced argmax of the full forward at every generated position
            ref = full[len(p) - 1:].argmax(-1).tolist()
            agree = sum(int(a == b) for a, b in zip(ref, s.output_ids)) / len(ref)
            assert agree >= 0.9, (graphs, agree)


def test_decode_logits_close_to_full_forward():
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama", dtype=torch.bfloat16, device=dev, init="random", seed=5)
    m.eval()
    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cuda", max_model_len=256,
                                 block_size=16, num_blocks=64, use_graphs=True), model=m)
    s = eng.add_request(list(range(10, 40)), SamplingParams(max_tokens=6, temperature=0,
                                                             ignore_eos=True))
    got = []
    orig = eng.runner.decode

    def spy(inp):
        out = orig(inp)
        got.append(out.float().clone())
        return out
    eng.runner.decode = spy
    while eng.has_work:
        eng.step()
    ids = torch.tensor([s.all_ids[:-1]], device=dev)
    with torch.no_grad():
        full = m(ids).float().view(ids.shape[1], -1)
    for k, lg in enumerate(got):
        ref = full[30 + k]
        rel = ((lg[0] - ref).norm() / ref.norm()).item()
        assert rel < 3e-2, (k, rel)


def test_multi_lora_graph_decode_matches_merged(tmp_path):
    """Un-merged adapters in hipGraph-captured decode vs an engine with the adapter merged."""
    from lumen.lora import LoraConfig, apply_lora, load_adapter, merge_lora, save_adapter
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)

    def base():
        m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
        with torch.no_grad():
            for p in m.parameters():
                if p.dim() == 2:
                    p.mul_(4.0)
        return m.eval()

    m = base()
    apply_lora(m, LoraConfig(r=16, lora_alpha=32))
    g = torch.Generator().manual_seed(7)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.requires_grad:
                p.copy_((torch.randn(p.shape, generator=g) * 0.2).to(dev))
    save_adapter(m, str(tmp_path / "ad"), "tiny-llama-gqa")
    prompts = [[5, 9, 33, 7] * 10, list(range(3, 60)), [42, 43]]
    sp = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True)
    multi = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=512,
                                   block_size=16, num_blocks=128, use_graphs=True,
                                   lora_modules={"ad": str(tmp_path / "ad")}), model=base())
    seqs = [multi.add_request(p, SamplingParams(**vars(sp)), lora="ad" if i != 1 else None)
            for i, p in enumerate(prompts)]
    while multi.has_work:
        multi.step()
    merged_m = base()
    load_adapter(merged_m, str(tmp_path / "ad"))
    merge_lora(merged_m)
    plain = base()
    for i, (p, s) in enumerate(zip(prompts, seqs)):
        ref_m = plain if i == 1 else merged_m
        ids = torch.tensor([p + s.output_ids[:-1]], device=dev)
        with torch.no_grad():
            full = ref_m(ids).float().view(ids.shape[1], -1)
        # teacher-forced argmax of the merged model at every generated position
        ref = full[len(p) - 1:].argmax(-1).tolist()
        agree = sum(int(a == b) for a, b in zip(ref, s.output_ids)) / len(ref)
        assert agree >= 0.85, (i, agree)


def test_prefix_caching_matches_full_forward():
    """Prompts sharing a 48-token prefix (3 blocks) on the HIP paged-prefill path: the later
    ones read the first one's cached K/V (published at its launch) and still agree with the
    full forward, teacher-forced."""
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
    m.eval()
    eng = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=512,
                                 block_size=16, num_blocks=128, use_graphs=True,
                                 scheduling_policy="prefill_first", max_num_batched_tokens=52,
                                 enable_prefix_caching=True), model=m)  # one prompt per step
    shared = [(7 * i + 3) % 500 for i in range(48)]
    prompts = [shared + [60 + i, 61, 62, 63 + i] for i in range(4)]
    seqs = [eng.add_request(p, SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True))
            for p in prompts]
    while eng.has_work:
        eng.step()
    assert eng.blocks.hit_tokens == 3 * 48
    for p, s in zip(prompts, seqs):
        ids = torch.tensor([p + s.output_ids[:-1]], device=dev)
        with torch.no_grad():
            full = m(ids).float().view(ids.shape[1], -1)
        ref = full[len(p) - 1:].argmax(-1).tolist()
        agree = sum(int(a == b) for a, b in zip(ref, s.output_ids)) / len(ref)
        assert agree >= 0.9, agree


def test_prompt_scores_and_alternatives_match_full_forward():
    """prompt_logprobs (echo scoring) and top_logprobs on the GPU path: the paged prefill's
    extra rows and the sampled rows against the full forward's log-softmax (bf16 tolerance)."""
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
    m.eval()
    eng = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=512,
                                 block_size=16, num_blocks=128, use_graphs=True,
                                 max_num_batched_tokens=32), model=m)   # chunked prompt
    prompt = [(11 * i + 5) % 500 for i in range(70)]
    s = eng.add_request(prompt, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True,
                                               top_logprobs=4, prompt_logprobs=3))
    while eng.has_work:
        eng.step()
    ids = torch.tensor([prompt + s.output_ids], device=dev)
    with torch.no_grad():
        lp = torch.log_softmax(m(ids).float().view(ids.shape[1], -1), -1)
    assert len(s.prompt_scores) == len(prompt) and s.prompt_scores[0] is None
    got = torch.tensor([x[0] for x in s.prompt_scores[1:]])
    ref = lp[torch.arange(len(prompt) - 1), torch.tensor(prompt[1:], device=dev)].cpu()
    assert (got - ref).abs().max().item() < 0.1, (got - ref).abs().max().item()
    assert len(s.output_top_logprobs) == 6
    for i, alts in enumerate(s.output_top_logprobs):
        row = lp[len(prompt) - 1 + i]
        assert abs(alts[0][1] - row.max().item()) < 0.1
        assert all(a[1] >= b[1] for a, b in zip(alts, alts[1:]))


def test_prompt_lookup_speculative_decoding_matches_full_forward():
    """Speculative verification on the GPU path (paged prefill over [last token | draft]
    chunks next to graph-free decode rows): teacher-forced agreement with the full forward."""
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
    m.eval()
    eng = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=512,
                                 block_size=16, num_blocks=128, use_graphs=True,
                                 num_speculative_tokens=4, spec_min_fraction=0.0),
                    model=m)   # verify every draft: exercise the GPU verify path
    prompts = [[5, 9, 33, 7] * 10, list(range(3, 60)) * 2, [42, 43]]
    seqs = [eng.add_request(p, SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True))
            for p in prompts]
    while eng.has_work:
        eng.step()
    assert eng.stats["spec_steps"] > 0
    for p, s in zip(prompts, seqs):
        assert len(s.output_ids) == 40
        ids = torch.tensor([p + s.output_ids[:-1]], device=dev)
        with torch.no_grad():
            full = m(ids).float().view(ids.shape[1], -1)
        ref = full[len(p) - 1:].argmax(-1).tolist()
        agree = sum(int(a == b) for a, b in zip(ref, s.output_ids)) / len(ref)
        assert agree >= 0.9, agree


@pytest.mark.parametrize("kv", ["auto", "fp8"])
def test_fresh_prompt_prefill_matches_paged(kv, monkeypatch):
    """Whole fresh prompts take flash attention straight from the q|k|v rows; the first-token
    logits equal the paged-cache prefill's (GQA tiny model, several prompts in one step)."""
    import lumen.serve.model_runner as mr
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
    m.eval()
    prompts = [list(range(3, 200)), [5, 9, 33, 7] * 20, list(range(100, 140))]

    def first_logits(fresh):
        monkeypatch.setattr(mr, "FRESH_PREFILL", fresh)
        eng = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=512,
                                     block_size=16, num_blocks=128, use_graphs=False,
                                     max_num_batched_tokens=1024, kv_cache_dtype=kv), model=m)
        got = []
        orig = eng.runner.execute

        def spy(inp):
            out = orig(inp)
            got.append(out.float().clone())
            return out
        eng.runner.execute = spy
        for p in prompts:
            eng.add_request(p, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
        while eng.has_work:
            eng.step()
        return got[0]

    a, b = first_logits(True), first_logits(False)
    assert a.shape == b.shape == (3, m.config.vocab_size)
    rel = ((a - b).norm() / b.norm()).item()
    # fp8: the paged path reads e4m3-rounded K/V, the fresh path the 16-bit rows
    assert rel < (2e-2 if kv == "auto" else 6e-2), rel


def test_split_decode_two_streams_matches(monkeypatch):
    """Decode batches run as two half-batches on two streams (LUMEN_DECODE_SPLIT; the second
    half forked after the first half's first projection, joined before the logits), eager and
    graph-captured: the decode logits equal the single-stream path's up to the bf16 rounding of
    the differently sized GEMMs, and the greedy tokens agree."""
    import lumen.serve.model_runner as mr
    from lumen.models import build_model
    from lumen.serve.engine import EngineConfig, LLMEngine
    from lumen.serve.sequence import SamplingParams

    dev = torch.device("cuda", 0)
    m = build_model("tiny-llama-gqa", dtype=torch.bfloat16, device=dev, init="random", seed=3)
    m.eval()
    g = torch.Generator().manual_seed(9)
    prompts = [torch.randint(3, 500, (int(n),), generator=g).tolist()
               for n in torch.randint(20, 60, (64,), generator=g)]

    def run(split, graphs):
        monkeypatch.setattr(mr, "DECODE_SPLIT_MIN", split)
        eng = LLMEngine(EngineConfig(model="tiny-llama-gqa", device="cuda", max_model_len=256,
                                     block_size=16, num_blocks=512, use_graphs=graphs,
                                     max_num_seqs=64, scheduling_policy="prefill_first",
                                     max_num_batched_tokens=8192), model=m)
        got = []
        orig = eng.runner.decode

        def spy(inp):
            out = orig(inp)
            if inp.tokens.shape[0] == 64:
                got.append(out.float().clone())
            return out
        eng.runner.decode = spy
        seqs = [eng.add_request(p, SamplingParams(max_tokens=6, temperature=0.0,
                                                  ignore_eos=True)) for p in prompts]
        while eng.has_work:
            eng.step()
        return [s.output_ids for s in seqs], got

    for graphs in (False, True):
        o0, l0 = run(0, graphs)
        o1, l1 = run(32, graphs)
        assert len(l0) == len(l1) and l0
        for a, b in zip(l0, l1):
            assert ((a - b).norm() / b.norm()).item() < 1e-2
        same = sum(int(x == y) for a, b in zip(o0, o1) for x, y in zip(a, b))
        assert same >= 0.95 * sum(len(a) for a in o0), (graphs, same)
