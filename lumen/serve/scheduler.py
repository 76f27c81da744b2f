"""Continuous-batching scheduler with chunked prefill and mixed prefill + decode steps
(the vLLM 0.6 engine the reference declares, README.md:10,16; re-designed).

Every engine step spends a TOKEN BUDGET (``max_num_batched_tokens``):

1. every running sequence that is past its prompt decodes one token (always: a prefill never
   stalls the running streams, which is what bounds inter-token latency under load); while
   only a few sequences decode, the budget is ``prefill_boost`` times larger (few streams pay
   for the longer step; a burst of arrivals reaches its first tokens sooner);
2. the rest of the budget goes to prefill CHUNKS, first to sequences whose prompt is already
   partly in the cache, then to waiting requests in arrival order.  A prompt longer than what
   is left is split: its first chunk runs now, the next chunks in later steps (its queries
   attend to the cached earlier chunks through the paged-prefill kernel).

The step is one forward over [prefill chunk tokens | decode tokens] (GEMMs see every token at
once); a sequence gets a sampled token only when the chunk that completes its prompt runs.
A step without prefill work is a pure decode step (hipGraph-captured in the runner).

``policy="prefill_first"`` is vLLM 0.6.0's default scheduling instead (the version the
reference pins; chunked prefill is opt-in there): while prompts wait and can be admitted, a step
is PREFILL-ONLY (whole prompts, FCFS, up to the token budget; only a prompt longer than the
budget is chunked); otherwise it is a decode step of every running sequence.  Prefills finish
sooner (higher throughput, lower TTFT under a burst) at the cost of a long pause in the running
streams while a burst is prefilled (its inter-token-latency maximum).

With prefix caching on (block_manager.py), admission shares the prompt's leading full blocks
that are already cached and only the rest of the prompt is prefilled.

KV blocks for a whole prompt are reserved when the request is admitted, so a chunked prefill
never runs out of blocks halfway; decodes grow their tables a block at a time, and when none is
left the youngest running sequence is preempted (blocks freed, requeued at the front, its prompt
plus the tokens generated so far recomputed on re-admission: vLLM's recompute preemption).
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Deque, List, Optional, Tuple

from .block_manager import BlockManager
from .sequence import Sequence, Status


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 2048
    max_model_len: int = 4096
    # prefill boost: while at most ``boost_max_decodes`` sequences are decoding, a step may
    # batch ``prefill_boost`` x the token budget.  The budget exists to bound the inter-token
    # latency of the running streams; with few of them, a longer step delays few tokens, and the
    # waiting prompts get their first token sooner (a burst of arrivals).  1 disables it.
    prefill_boost: int = 1
    boost_max_decodes: int = 0   # 0: max_num_seqs // 4
    policy: str = "chunked"      # "chunked" (mixed steps) | "prefill_first" (vLLM 0.6 default)


@dataclass
class Batch:
    kind: str          # "mixed" | "decode" | "verify" (speculative drafts, engine-built)
    prefills: List[Tuple[Sequence, int]] = field(default_factory=list)  # (seq, chunk length)
    decodes: List[Sequence] = field(default_factory=list)

    @property
    def seqs(self) -> List[Sequence]:
        return [s for s, _ in self.prefills] + self.decodes

    @property
    def num_tokens(self) -> int:
        return sum(c for _, c in self.prefills) + len(self.decodes)

    def completing(self) -> List[Sequence]:
        """Prefill sequences whose prompt this step finishes (they get a sampled token)."""
        return [s for s, c in self.prefills if s.num_cached + c == s.length]

    @property
    def sampled(self) -> List[Sequence]:
        """Rows of the step's logits, in order: completing prefills, then decodes."""
        return self.completing() + self.decodes


class Scheduler:
    POLICIES = ("chunked", "prefill_first")

    def __init__(self, cfg: SchedulerConfig, blocks: BlockManager):
        if cfg.policy not in self.POLICIES:
            raise ValueError(f"scheduling policy must be one of {self.POLICIES}, got {cfg.policy!r}")
        self.cfg = cfg
        self.blocks = blocks
        self.waiting: Deque[Sequence] = deque()
        self.running: List[Sequence] = []
        self.num_preemptions = 0

    def add(self, seq: Sequence) -> None:
        if seq.length > self.cfg.max_model_len:
            raise ValueError(f"prompt of {seq.length} tokens exceeds max_model_len "
                             f"{self.cfg.max_model_len}")
        self.waiting.append(seq)

    def abort(self, request_id: str) -> None:
        for q in (self.waiting, self.running):
            for s in list(q):
                if s.request_id == request_id:
                    q.remove(s)
                    s.status, s.finish_reason = Status.FINISHED, "abort"
                    self.blocks.free_seq(s.seq_id)

    @property
    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def _admit(self, batch: Batch, budget: int, skip=()) -> int:
        """Prefill work into ``batch``: partially cached prompts first, then waiting requests in
        arrival order, while the token budget, ``max_num_seqs`` and the free blocks allow."""
        for s in self.running:
            if budget <= 0:
                break
            if not s.prefilled and s.seq_id not in skip:
                c = min(s.length - s.num_cached, budget)
                batch.prefills.append((s, c))
                budget -= c
        whole = self.cfg.policy == "prefill_first"
        share = self.blocks.prefix_caching
        pending = set()   # first blocks this batch computes (named when it is launched)
        while self.waiting and budget > 0 and len(self.running) < self.cfg.max_num_seqs:
            s = self.waiting[0]
            if not self.blocks.can_allocate(s.length + 1):
                break
            if whole and batch.prefills and not self._fits(s, budget):
                break   # vLLM 0.6 (no chunked prefill): whole prompts only, FCFS
            d0 = self._first_block(s) if share else None
            if d0 is not None and d0 in pending and s.params.prompt_logprobs is None:
                # the same prompt start is being computed by this step (n > 1 choices, a
                # shared system prompt): wait one step and share its blocks instead
                break
            self.waiting.popleft()
            # prefix caching: the leading full blocks already in the cache are shared and only
            # the rest of the prompt is computed (0 without it)
            # (a prompt to be scored is computed whole: no shared blocks)
            s.num_cached = self.blocks.allocate(
                s.seq_id, s.length + 1,
                s.all_ids if s.params.prompt_logprobs is None else None, s.lora_slot)
            s.prefilled = False
            s.status = Status.RUNNING
            self.running.append(s)
            c = min(s.length - s.num_cached, budget)
            batch.prefills.append((s, c))
            budget -= c
            if d0 is not None and s.num_cached == 0:
                pending.add(d0)
        return budget

    def _first_block(self, s: Sequence):
        """Name of the sequence's first full block (None if its prompt has none to share)."""
        bs = self.blocks.block_size
        if s.length - 1 < bs:
            return None
        from .block_manager import block_digest
        return block_digest(b"", s.lora_slot, s.all_ids[:bs])

    def _fits(self, s: Sequence, budget: int) -> bool:
        """Would ``s``'s whole uncached prompt fit ``budget``?  (Prefix-cache hits are counted
        only by looking the blocks up; the allocation itself happens at admission.)"""
        if s.length <= budget:
            return True
        bm = self.blocks
        if not bm.prefix_caching or s.params.prompt_logprobs is not None:
            return False
        ids = s.all_ids
        hit = 0
        for d in bm._digests(ids, (len(ids) - 1) // bm.block_size, s.lora_slot):
            if d not in bm.cached:
                break
            hit += bm.block_size
        return s.length - hit <= budget

    def schedule(self) -> Optional[Batch]:
        budget = self.cfg.max_num_batched_tokens
        batch = Batch("mixed")
        if self.cfg.policy == "prefill_first":
            # vLLM 0.6: a prefill-only step whenever prompt work can be scheduled
            self._admit(batch, budget)
            if batch.prefills:
                return batch
        # 1) one token for every sequence past its prompt (grow block tables; preempt the
        #    youngest running sequence when the cache is exhausted)
        preempted = set()
        for s in list(self.running):
            if s.seq_id in preempted or not s.prefilled or s.capped:
                continue
            while True:
                try:
                    self.blocks.ensure(s.seq_id, s.length + 1)
                    batch.decodes.append(s)
                    break
                except RuntimeError:
                    victim = self.running[-1]
                    self._preempt(victim)
                    preempted.add(victim.seq_id)
                    if victim in batch.decodes:
                        batch.decodes.remove(victim)
                    if victim is s:
                        break
        if self.cfg.prefill_boost > 1 and len(batch.decodes) <= (
                self.cfg.boost_max_decodes or self.cfg.max_num_seqs // 4):
            budget *= self.cfg.prefill_boost
        budget -= len(batch.decodes)
        # 2) continue partially cached prompts, then admit waiting requests (FCFS); the
        #    prefill-first policy reaches here only for decode steps
        if self.cfg.policy != "prefill_first":
            self._admit(batch, budget, skip=preempted)
        if not batch.prefills and not batch.decodes:
            return None
        if not batch.prefills:
            batch.kind = "decode"
        return batch

    def launched(self, batch: Batch) -> None:
        """The engine launched ``batch`` (before it advances ``num_cached``): with prefix
        caching, the full prompt blocks its prefill chunks write become shareable."""
        if self.blocks.prefix_caching:
            for s, c in batch.prefills:
                self.blocks.publish(s.seq_id, s.all_ids, s.num_cached + c, s.lora_slot)

    def _release(self, s: Sequence) -> None:
        """Free a retired / preempted sequence's blocks; with prefix caching its full blocks
        whose K/V launched steps wrote stay cached (a recomputed or follow-up prompt hits them)."""
        self.blocks.free_seq(s.seq_id, s.all_ids, min(s.num_cached, len(s.all_ids)),
                             s.lora_slot)

    def _preempt(self, s: Sequence) -> None:
        self.running.remove(s)
        self._release(s)
        s.status = Status.WAITING
        s.num_cached = 0
        s.prefilled = False
        s.preemptions += 1
        self.num_preemptions += 1
        # recompute: re-admission prefills prompt + tokens generated so far (outputs kept, so
        # streaming clients see no duplicate tokens)
        self.waiting.appendleft(s)

    def finish(self, batch: Batch) -> List[Sequence]:
        return self.finish_seqs(batch.seqs)

    def finish_seqs(self, seqs) -> List[Sequence]:
        """Retire the finished ones among ``seqs`` (running list, KV blocks)."""
        live = {s.seq_id for s in self.running}
        done = [s for s in seqs if s.finished and s.seq_id in live]
        if done:
            ids = {s.seq_id for s in done}
            self.running = [s for s in self.running if s.seq_id not in ids]
            for s in done:
                self._release(s)
        return done
