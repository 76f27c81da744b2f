"""Automatic prefix caching (vLLM --enable-prefix-caching semantics; lumen/serve/block_manager.py):
block naming, sharing, publication on finish, LRU eviction; and engine runs on CPU whose greedy
outputs must equal full-recompute decoding while prompts reuse cached K/V."""
import pytest
import torch

from lumen.models import build_model
from lumen.serve.block_manager import BlockManager
from lumen.serve.engine import EngineConfig, LLMEngine
from lumen.serve.sequence import SamplingParams


# ---------------------------------------------------------------------------------------------
# block manager


def test_hits_are_whole_leading_blocks_and_leave_one_token():
    bm = BlockManager(32, 4, watermark=0.0, prefix_caching=True)
    ids = list(range(100, 113))                     # 13 tokens: 3 full blocks + 1
    assert bm.allocate(1, len(ids) + 1, ids) == 0   # cold cache
    bm.free_seq(1, ids, n_computed=len(ids))
    assert len(bm.parked) == 3 and bm.num_free == 32
    assert bm.allocate(2, len(ids) + 1, ids) == 12  # 3 blocks shared
    # a prompt of exactly 3 full blocks computes its last block again (its logits are needed)
    assert bm.allocate(3, 13, ids[:12]) == 8
    # a different first block: no hit at all (names chain the whole prefix)
    assert bm.allocate(4, 14, [7] + ids[1:]) == 0
    # another adapter slot: no hit
    assert bm.allocate(5, 14, ids, lora=2) == 0
    t2, t3 = bm.tables[2], bm.tables[3]
    assert t2[:2] == t3[:2] and bm.ref[t2[0]] == 2 and bm.ref[t2[2]] == 1
    for sid in (2, 3, 4, 5):
        bm.free_seq(sid)
    assert bm.num_free == 32 and not bm.ref
    assert bm.hit_tokens == 20 and bm.query_tokens == 13 * 4 + 12


def test_only_computed_blocks_are_published_and_duplicates_released():
    bm = BlockManager(16, 4, watermark=0.0, prefix_caching=True)
    ids = list(range(10))
    bm.allocate(1, 11, ids)
    bm.free_seq(1, ids, n_computed=5)               # K/V written for 5 tokens: 1 full block
    assert len(bm.parked) == 1
    bm.allocate(2, 11, ids)
    bm.allocate(3, 11, ids)                          # both share block 0, compute block 1 twice
    bm.free_seq(2, ids, n_computed=10)
    bm.free_seq(3, ids, n_computed=10)               # its block 1 duplicates seq 2's: released
    assert len(bm.parked) == 2 and len(bm.cached) == 2
    assert bm.num_free == 16
    bm.reset_prefix_cache()
    assert not bm.cached and not bm.parked and bm.num_free == 16


def test_reset_never_publishes_blocks_computed_before_it():
    """A sequence running across ``reset_prefix_cache`` holds K/V of the old weights: freeing it
    afterwards must not name its blocks."""
    bm = BlockManager(16, 4, watermark=0.0, prefix_caching=True)
    ids = list(range(10))
    bm.allocate(1, 11, ids)
    bm.reset_prefix_cache()
    bm.free_seq(1, ids, n_computed=10)
    assert not bm.cached and not bm.parked and bm.num_free == 16
    assert bm.allocate(2, 11, ids) == 0              # no hit on pre-reset content
    bm.free_seq(2, ids, n_computed=10)               # a post-reset sequence publishes again
    assert len(bm.cached) == 2 and not bm.stale


def test_eviction_is_lru_and_tail_first():
    bm = BlockManager(5, 2, watermark=0.0, prefix_caching=True)
    a, b = [1, 2, 3, 4, 5], [6, 7, 8, 9, 10, 11, 12]
    bm.allocate(1, 5, a)
    bm.free_seq(1, a, n_computed=5)                  # a's 2 full blocks parked, tail first
    bm.allocate(2, 7, b)                             # 3 unnamed free blocks + evicts a's tail
    assert len(bm.parked) == 1
    bm.free_seq(2)
    assert bm.allocate(3, 5, a) == 2                 # a's head block survived
    bm.free_seq(3)
    assert bm.num_free == 5 and not bm.ref


# ---------------------------------------------------------------------------------------------
# engine


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


def _engine(model, **kw):
    cfg = EngineConfig(model="tiny-llama-gqa", device="cpu", max_model_len=256, block_size=4,
                       use_graphs=False, enable_prefix_caching=True, **kw)
    return LLMEngine(cfg, model=model)


GREEDY = dict(temperature=0.0, ignore_eos=True)
SYSTEM = [31, 7, 99, 12, 5, 64, 3, 8, 41, 17, 23, 2, 77]   # a shared 13-token "system prompt"


@pytest.mark.parametrize("policy,async_sched", [("prefill_first", True), ("prefill_first", False),
                                                ("chunked", True)])
def test_shared_prefix_requests_match_naive(model, policy, async_sched):
    eng = _engine(model, num_blocks=256, scheduling_policy=policy,
                  async_scheduling=async_sched, max_num_batched_tokens=64)
    first = SYSTEM + [50, 51]
    s0 = eng.generate([first], SamplingParams(max_tokens=6, **GREEDY))[0]
    assert s0.output_ids == naive_greedy(model, first, 6)
    prompts = [SYSTEM + [60 + i, 61 + i, 62] for i in range(4)] + [SYSTEM[:9]]
    seqs = eng.generate(prompts, SamplingParams(max_tokens=8, **GREEDY))
    for p, s in zip(prompts, seqs):
        assert s.output_ids == naive_greedy(model, p, 8), p
    # every later prompt reused the system prompt's 3 full blocks (the short one 2)
    assert eng.blocks.hit_tokens == 4 * 12 + 8
    assert eng.blocks.num_free == eng.blocks.num_blocks
    assert eng.stats["prefill_tokens"] == len(first) + sum(len(p) for p in prompts) - 56


def test_multi_turn_reuses_previous_answer(model):
    eng = _engine(model, num_blocks=256, scheduling_policy="prefill_first")
    turn1 = SYSTEM + [90, 91, 92]
    s1 = eng.generate([turn1], SamplingParams(max_tokens=9, **GREEDY))[0]
    turn2 = turn1 + s1.output_ids + [93, 94]
    before = eng.blocks.hit_tokens
    s2 = eng.generate([turn2], SamplingParams(max_tokens=7, **GREEDY))[0]
    assert s2.output_ids == naive_greedy(model, turn2, 7)
    # K/V of turn 1's prompt + all but its last answer token were written: 24 tokens -> 6 blocks
    assert eng.blocks.hit_tokens - before == 24


def test_prefix_cache_under_preemption_and_eviction(model):
    """Too few blocks for the running streams: preemption publishes the victim's computed
    blocks, recompute hits them, distinct prompts evict parked blocks -- outputs unchanged."""
    eng = _engine(model, num_blocks=16, scheduling_policy="prefill_first",
                  max_num_batched_tokens=64)
    eng.blocks.watermark_blocks = 0
    prompts = [SYSTEM[:4] + [3, 4, 5, 6], SYSTEM[:4] + [9, 10, 11, 12],
               [20, 21, 22, 23, 24, 25, 26, 27], [40, 41, 42, 43]]
    seqs = eng.generate(prompts, SamplingParams(max_tokens=20, **GREEDY))
    assert eng.scheduler.num_preemptions > 0
    for p, s in zip(prompts, seqs):
        assert s.output_ids == naive_greedy(model, p, 20), p
    assert eng.blocks.num_free == eng.blocks.num_blocks and not eng.blocks.ref


def test_prefix_caching_off_by_default(model):
    cfg = EngineConfig(model="tiny-llama-gqa", device="cpu", max_model_len=256, block_size=4,
                       use_graphs=False, num_blocks=64)
    eng = LLMEngine(cfg, model=model)
    for _ in range(2):
        eng.generate([SYSTEM + [1, 2]], SamplingParams(max_tokens=3, **GREEDY))
    assert eng.blocks.hit_tokens == 0 and not eng.blocks.cached


@pytest.mark.parametrize("async_sched", [True, False])
def test_burst_shares_prompt_blocks_published_at_launch(model, async_sched):
    """One burst, one prompt admitted per step: prompt blocks are named when their prefill is
    launched, so every later admission of the burst already shares them."""
    eng = _engine(model, num_blocks=256, scheduling_policy="prefill_first",
                  async_scheduling=async_sched, max_num_batched_tokens=16)
    prompts = [SYSTEM + [70 + i, 71, 72] for i in range(5)]    # 16 tokens each
    seqs = eng.generate(prompts, SamplingParams(max_tokens=5, **GREEDY))
    for p, s in zip(prompts, seqs):
        assert s.output_ids == naive_greedy(model, p, 5), p
    assert eng.blocks.hit_tokens == 4 * 12
    assert eng.blocks.num_free == eng.blocks.num_blocks


def test_abort_releases_shared_blocks(model):
    """Aborting requests that share cached blocks (waiting and running) drops only their
    references: the cache stays valid for the others and every block comes back."""
    eng = _engine(model, num_blocks=128, scheduling_policy="prefill_first")
    eng.generate([SYSTEM + [1, 2]], SamplingParams(max_tokens=2, **GREEDY))
    a = eng.add_request(SYSTEM + [3, 4], SamplingParams(max_tokens=30, **GREEDY), "a")
    b = eng.add_request(SYSTEM + [5, 6], SamplingParams(max_tokens=8, **GREEDY), "b")
    for _ in range(3):
        eng.step()
    eng.abort("a")
    c = eng.add_request(SYSTEM + [7], SamplingParams(max_tokens=4, **GREEDY), "c")
    eng.abort("c")                                   # aborted while waiting
    while eng.has_work:
        eng.step()
    assert b.output_ids == naive_greedy(model, SYSTEM + [5, 6], 8)
    assert a.finish_reason == "abort" and c.finish_reason == "abort"
    assert eng.blocks.num_free == eng.blocks.num_blocks and not eng.blocks.ref


@pytest.mark.parametrize("policy", ["prefill_first", "chunked"])
def test_same_step_duplicates_wait_and_share(model, policy):
    """A burst whose prompts start alike, all fitting one step: the first computes the shared
    blocks, the rest wait one step and share them (n > 1 choices, a common system prompt)."""
    eng = _engine(model, num_blocks=256, scheduling_policy=policy,
                  max_num_batched_tokens=256)
    prompts = [SYSTEM + [80 + i] for i in range(4)] + [SYSTEM + [80]] * 2   # 14 tokens each
    seqs = eng.generate(prompts, SamplingParams(max_tokens=5, **GREEDY))
    for p, s in zip(prompts, seqs):
        assert s.output_ids == naive_greedy(model, p, 5), p
    assert eng.blocks.hit_tokens == 5 * 12        # 3 full blocks, shared by the 5 later ones
    assert eng.blocks.num_free == eng.blocks.num_blocks
