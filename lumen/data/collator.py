"""Causal-LM collation.

Matches transformers' DataCollatorForLanguageModeling(mlm=False) as used by the reference
(training/train_baseline.py:195-198): pad to the longest sequence in the batch with the pad id
(pad = eos, training/train_baseline.py:116-117), labels = input_ids with pad positions set to
-100 -- so, as in the reference, a genuine EOS equal to pad is masked too
when ``mask_pad_equal_eos`` is True.

lumen's model consumes labels already shifted by one (label[t] = token[t+1]), so the loss kernel
runs over all T positions with no slicing copy; ``n_valid`` (count of non-ignored labels) is
computed here on the host so the loss normalisation needs no device sync.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

IGNORE = -100


def shift_labels(labels: torch.Tensor) -> torch.Tensor:
    out = torch.full_like(labels, IGNORE)
    out[:, :-1] = labels[:, 1:]
    return out


class CausalLMCollator:
    def __init__(self, pad_id: int, max_length: Optional[int] = None, pad_to_multiple_of: int = 1,
                 mask_pad_equal_eos: bool = True, fixed_length: Optional[int] = None):
        self.pad_id = pad_id
        self.max_length = max_length
        self.mult = max(1, pad_to_multiple_of)
        self.mask_pad = mask_pad_equal_eos
        self.fixed_length = fixed_length

    def __call__(self, examples: Sequence) -> Dict[str, torch.Tensor]:
        seqs: List[List[int]] = []
        for e in examples:
            ids = e["input_ids"] if isinstance(e, dict) else e
            ids = list(ids)
            if self.max_length:
                ids = ids[: self.max_length]
            seqs.append(ids)
        L = self.fixed_length or max(len(s) for s in seqs)
        L = (L + self.mult - 1) // self.mult * self.mult
        B = len(seqs)
        input_ids = torch.full((B, L), self.pad_id, dtype=torch.long)
        attn = torch.zeros((B, L), dtype=torch.long)
        for i, s in enumerate(seqs):
            n = min(len(s), L)
            input_ids[i, :n] = torch.tensor(s[:n], dtype=torch.long)
            attn[i, :n] = 1
        labels = input_ids.clone()
        if self.mask_pad:
            labels[input_ids == self.pad_id] = IGNORE
        labels[attn == 0] = IGNORE
        shifted = shift_labels(labels)
        n_valid = int((shifted != IGNORE).sum())
        n_tokens = int(attn.sum())
        return {"input_ids": input_ids, "labels": shifted, "attention_mask": attn,
                "n_valid": n_valid, "n_tokens": n_tokens}
