"""Request / sequence state for the serving engine."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import List, Optional, Tuple


@dataclass
class SamplingParams:
    max_tokens: int = 16
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0            # 0 = disabled
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None
    logprobs: bool = False
    # OpenAI / vLLM logprobs: alternatives per generated token (the most likely ``top_logprobs``
    # tokens of the distribution the token was sampled from), and prompt_logprobs (None: off):
    # the log probability of every prompt token given its prefix plus that many alternatives
    # (``echo`` scoring; TP = 1)
    top_logprobs: int = 0
    prompt_logprobs: Optional[int] = None
    # OpenAI penalties (logit -= frequency * count + presence * [count > 0], over the generated
    # tokens) and vLLM's repetition penalty (prompt + generated tokens: positive logits divided,
    # negative multiplied)
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0

    @property
    def has_penalties(self) -> bool:
        return (self.presence_penalty != 0.0 or self.frequency_penalty != 0.0
                or self.repetition_penalty != 1.0)

    def __post_init__(self):
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if not -2.0 <= self.presence_penalty <= 2.0 or not -2.0 <= self.frequency_penalty <= 2.0:
            raise ValueError("presence_penalty / frequency_penalty must be in [-2, 2]")
        if self.repetition_penalty <= 0:
            raise ValueError("repetition_penalty must be > 0")
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0.0 < self.top_p <= 1.0:
            raise ValueError("top_p must be in (0, 1]")
        if not 0 <= self.top_logprobs <= 20:
            raise ValueError("top_logprobs must be in [0, 20]")
        if self.prompt_logprobs is not None and not 0 <= self.prompt_logprobs <= 20:
            raise ValueError("prompt_logprobs must be in [0, 20]")

    @property
    def wants_extras(self) -> bool:
        """Alternatives or prompt scores: the step is resolved on the host before the next."""
        return self.top_logprobs > 0 or self.prompt_logprobs is not None


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


_ids = itertools.count()


PENDING = -1  # last_token of a sequence whose next input token is still on the device


@dataclass
class Sequence:
    prompt_ids: List[int]
    params: SamplingParams
    request_id: str = ""
    seq_id: int = field(default_factory=lambda: next(_ids))
    output_ids: List[int] = field(default_factory=list)
    output_logprobs: List[float] = field(default_factory=list)
    # per generated token: [(token id, logprob)] of the top_logprobs alternatives
    output_top_logprobs: List[List[Tuple[int, float]]] = field(default_factory=list)
    # prompt_logprobs: per prompt token (None for the first), (logprob, alternatives)
    prompt_scores: List[Optional[Tuple[float, List[Tuple[int, float]]]]] = field(
        default_factory=list)
    status: Status = Status.WAITING
    finish_reason: Optional[str] = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    last_token_time: Optional[float] = None
    token_times: List[float] = field(default_factory=list)
    num_cached: int = 0          # tokens whose K/V are in the cache
    prefilled: bool = False      # prompt (incl. recomputed outputs) fully in the cache
    preemptions: int = 0
    lora_slot: int = 0           # multi-LoRA serving: adapter slot (0 = base model)
    n_pending: int = 0           # async scheduling: sampled tokens still on the device
    capped: bool = False         # max_tokens reached counting in-flight tokens
    draft: List[int] = field(default_factory=list)   # speculative tokens under verification
    spec_wait: int = 0           # decode steps before this sequence drafts again (back-off)
    spec_misses: int = 0         # consecutive verifications that accepted nothing
    # prompt lookup: n-gram -> position after its latest occurrence, over all_ids[:ngram_upto]
    ngram_idx: dict = field(default_factory=dict, repr=False)
    ngram_upto: int = 0

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    @property
    def length(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids) + self.n_pending

    @property
    def last_token(self) -> int:
        if self.n_pending:
            return PENDING
        return self.output_ids[-1] if self.output_ids else self.prompt_ids[-1]

    @property
    def finished(self) -> bool:
        return self.status == Status.FINISHED

    def reserve(self) -> None:
        """Async scheduling: a step that samples this sequence's next token is in flight.
        Lengths / block tables count it now; ``output_ids`` only ever holds resolved tokens (a
        streaming reader on another thread never sees a placeholder).  A sequence whose
        max_tokens the in-flight tokens reach is ``capped``: no further steps are scheduled."""
        self.n_pending += 1
        if len(self.output_ids) + self.n_pending >= self.params.max_tokens:
            self.capped = True

    def fill(self, tok: int, logprob: Optional[float], eos_id: Optional[int]) -> None:
        """The value of the oldest in-flight token (resolved in launch order)."""
        now = time.perf_counter()
        if self.first_token_time is None:
            self.first_token_time = now
        self.last_token_time = now
        self.token_times.append(now)
        if logprob is not None:
            self.output_logprobs.append(logprob)
        self.output_ids.append(tok)
        self.n_pending -= 1
        p = self.params
        if (not p.ignore_eos and eos_id is not None and tok == eos_id) or tok in p.stop_token_ids:
            self.status, self.finish_reason = Status.FINISHED, "stop"
        elif len(self.output_ids) >= p.max_tokens:
            self.status, self.finish_reason = Status.FINISHED, "length"

    @property
    def has_pending(self) -> bool:
        return self.n_pending > 0

    def append(self, tok: int, logprob: Optional[float], eos_id: Optional[int],
               top: Optional[List[Tuple[int, float]]] = None) -> None:
        if top is not None:
            self.output_top_logprobs.append(top)
        now = time.perf_counter()
        if self.first_token_time is None:
            self.first_token_time = now
        self.last_token_time = now
        self.token_times.append(now)
        self.output_ids.append(tok)
        if logprob is not None:
            self.output_logprobs.append(logprob)
        p = self.params
        if not p.ignore_eos and eos_id is not None and tok == eos_id:
            self.status, self.finish_reason = Status.FINISHED, "stop"
        elif tok in p.stop_token_ids:
            self.status, self.finish_reason = Status.FINISHED, "stop"
        elif len(self.output_ids) >= p.max_tokens:
            self.status, self.finish_reason = Status.FINISHED, "length"
