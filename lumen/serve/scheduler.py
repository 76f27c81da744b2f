"""Continuous-batching scheduler (vLLM 0.6 semantics, re-designed).

Every engine step is either a PREFILL step (admit waiting requests while the token budget and
free KV blocks allow; their whole prompts run as one packed batch) or a DECODE step (one token
for every running sequence).  Prefill has priority, as in vLLM's default policy, which keeps
TTFT low under load; decode batches grow and shrink every step as requests join and finish.
When a decode step cannot get a new KV block the youngest running sequence is preempted
(blocks freed, sequence requeued at the front, recomputed on re-admission).
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Deque, List, Optional

from .block_manager import BlockManager
from .sequence import Sequence, Status


@dataclass
class SchedulerConfig:
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 16384
    max_model_len: int = 4096


@dataclass
class Batch:
    kind: str                       # "prefill" | "decode"
    seqs: List[Sequence] = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        if self.kind == "decode":
            return len(self.seqs)
        return sum(s.length - s.num_cached for s in self.seqs)


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, blocks: BlockManager):
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

    def schedule(self) -> Optional[Batch]:
        # 1) prefill: admit in FCFS order while budget / blocks / seq slots allow
        if self.waiting:
            batch = Batch("prefill")
            budget = self.cfg.max_num_batched_tokens
            while self.waiting and len(self.running) + len(batch.seqs) < self.cfg.max_num_seqs:
                s = self.waiting[0]
                n = s.length
                if batch.seqs and n > budget:
                    break
                if not self.blocks.can_allocate(n + 1):
                    break
                self.waiting.popleft()
                self.blocks.allocate(s.seq_id, n + 1)
                s.num_cached = 0
                s.status = Status.RUNNING
                batch.seqs.append(s)
                budget -= n
            if batch.seqs:
                self.running.extend(batch.seqs)
                return batch
        # 2) decode every running sequence (grow block tables; preempt on exhaustion)
        if not self.running:
            return None
        ready: List[Sequence] = []
        preempted = set()
        for s in list(self.running):
            if s.seq_id in preempted:
                continue
            while True:
                try:
                    self.blocks.ensure(s.seq_id, s.length + 1)
                    ready.append(s)
                    break
                except RuntimeError:
                    victim = self.running[-1]
                    self._preempt(victim)
                    preempted.add(victim.seq_id)
                    if victim is s:
                        break
                    if victim in ready:
                        ready.remove(victim)
        if not ready:
            return None
        return Batch("decode", ready)

    def _preempt(self, s: Sequence) -> None:
        self.running.remove(s)
        self.blocks.free_seq(s.seq_id)
        s.status = Status.WAITING
        s.num_cached = 0
        s.preemptions += 1
        self.num_preemptions += 1
        # recompute: re-admission prefills prompt + tokens generated so far (outputs kept, so
        # streaming clients see no duplicate tokens)
        self.waiting.appendleft(s)

    def finish(self, batch: Batch) -> List[Sequence]:
        done = [s for s in batch.seqs if s.finished]
        if done:
            ids = {s.seq_id for s in done}
            self.running = [s for s in self.running if s.seq_id not in ids]
            for s in done:
                self.blocks.free_seq(s.seq_id)
        return done
