"""Loss / perplexity and generation evaluation loops (see lumen/eval/__init__.py)."""
from __future__ import annotations

import math
import re
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..data.sampler import ShardedSampler
from .metrics import score_pairs

_CHAT = re.compile(r"^\s*(?:<s>)?\s*\[INST\]\s*(.*?)\s*\[/INST\]\s*(.*?)\s*(?:</s>)?\s*$", re.S)


def split_llama2_chat(text: str) -> Tuple[str, str]:
    """``<s>[INST] q [/INST] a</s>`` -> (``<s>[INST] q [/INST]``, ``a``); other text -> (text, "")."""
    m = _CHAT.match(text)
    if not m:
        return text, ""
    return f"<s>[INST] {m.group(1)} [/INST]", m.group(2)


@torch.no_grad()
def evaluate_loss(model, dataset, collator, batch_size: int = 8, device=None,
                  rank: int = 0, world: int = 1, group=None,
                  max_batches: Optional[int] = None) -> Dict[str, float]:
    """Token-weighted mean loss over ``dataset`` (each rank takes a strided shard; the
    padded tail of the last shard is excluded), plus perplexity = exp(loss)."""
    was_training = model.training
    model.eval()
    device = device or next(model.parameters()).device
    sampler = ShardedSampler(len(dataset), rank, world, shuffle=False)
    idx = [i for i in sampler.indices(0)]
    # the sampler pads every shard to the same length by repeating the head; drop the repeats
    seen = rank + world * torch.arange(len(idx))
    idx = [i for i, s in zip(idx, seen.tolist()) if s < len(dataset)]
    tot = torch.zeros(2, dtype=torch.float64, device=device)
    nb = 0
    for b0 in range(0, len(idx), batch_size):
        if max_batches is not None and nb >= max_batches:
            break
        batch = collator([dataset[i] for i in idx[b0:b0 + batch_size]])
        nv = int(batch["n_valid"])
        if nv == 0:
            continue
        loss = model(batch["input_ids"].to(device), batch["labels"].to(device), nv)
        tot[0] += loss.double() * nv
        tot[1] += nv
        nb += 1
    if world > 1 and dist.is_initialized():
        dist.all_reduce(tot, group=group)
    if was_training:
        model.train()
    s, n = float(tot[0]), float(tot[1])
    mean = s / n if n else float("nan")
    return {"eval_loss": mean, "perplexity": math.exp(min(mean, 80.0)) if n else float("nan"),
            "eval_tokens": int(n)}


def evaluate_generation(engine, prompts: Sequence[str], references: Sequence[str],
                        max_new_tokens: int = 128) -> Dict[str, object]:
    """Greedy completions of ``prompts`` through ``engine`` (an ``LLMEngine``), scored against
    ``references``.  Returns the mean metrics and the individual predictions."""
    from ..serve.sequence import SamplingParams

    params = SamplingParams(max_tokens=max_new_tokens, temperature=0.0)
    seqs = engine.generate(list(prompts), params)
    tok = engine.tokenizer
    preds: List[str] = [tok.decode(s.output_ids, skip_special_tokens=True) for s in seqs]
    metrics = score_pairs(zip(preds, references))
    return {"metrics": metrics, "predictions": preds}
