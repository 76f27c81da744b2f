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
