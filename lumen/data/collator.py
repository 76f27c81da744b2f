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


def fuse_collated(cbs: Sequence[Dict]) -> Dict:
    """Concatenate collated micro-batches into one batch (gradient-accumulation fusion).

    Packed batches join end to end (``cu_seqlens`` shifted; every part is already padded to the
    tuned multiple, so the sum stays on the grid); padded batches are re-padded to the longest
    row and stacked.  ``micro_steps`` tells the engine how many accumulation micro-steps the
    batch stands for."""
    if len(cbs) == 1:
        return dict(cbs[0], micro_steps=1)
    out: Dict = {"n_valid": sum(c["n_valid"] for c in cbs),
                 "n_tokens": sum(c["n_tokens"] for c in cbs), "micro_steps": len(cbs)}
    if cbs[0].get("cu_seqlens") is not None:
        cu, o = [0], 0
        for c in cbs:
            cu += [o + x for x in c["cu_seqlens"][1:]]
            o += c["input_ids"].shape[1]
        out.update(input_ids=torch.cat([c["input_ids"] for c in cbs], 1),
                   labels=torch.cat([c["labels"] for c in cbs], 1),
                   pos=torch.cat([c["pos"] for c in cbs]), cu_seqlens=tuple(cu),
                   n_padded=o, n_seqs=sum(c.get("n_seqs", 0) for c in cbs))
        return out
    L = max(c["input_ids"].shape[1] for c in cbs)

    def pad(t, v):
        return torch.nn.functional.pad(t, (0, L - t.shape[1]), value=v)

    # right padding under causal attention: the filler id is never attended to by a real token
    # and never a target, so any id works
    out.update(input_ids=torch.cat([pad(c["input_ids"], 0) for c in cbs]),
               labels=torch.cat([pad(c["labels"], IGNORE) for c in cbs]),
               attention_mask=torch.cat([pad(c["attention_mask"], 0) for c in cbs]))
    return out


class PackedCollator:
    """Sequence packing for the varlen flash-attention path (no padding compute).

    The micro-batch's sequences are laid back to back in ONE row of T = sum(len) tokens;
    ``cu_seqlens`` marks their boundaries so attention stays within each sequence, and
    ``pos`` restarts RoPE positions at 0 per sequence.  Labels are shifted WITHIN each sequence
    (the last token of a sequence predicts nothing), and -- as in the padded collator / the
    reference's DataCollatorForLanguageModeling with pad = eos -- a token equal to the pad id
    is never a target.  The loss over the packed row therefore equals the padded batch's
    (mean over the same valid labels), at sum(len) instead of B * max(len) tokens.

    T is rounded up to ``pad_to_multiple_of`` (default 256) so the frozen-weight GEMMs meet a
    small set of M values that the tuned hipBLASLt table covers; the filler tokens form one
    extra sequence of their own (attends only to itself, no labels)."""

    def __init__(self, pad_id: int, max_length: Optional[int] = None, pad_to_multiple_of: int = 256,
                 mask_pad_equal_eos: bool = True):
        self.pad_id = pad_id
        self.max_length = max_length
        self.mult = max(1, pad_to_multiple_of)
        self.mask_pad = mask_pad_equal_eos

    def __call__(self, examples: Sequence) -> Dict:
        import numpy as np

        seqs = []
        for e in examples:
            ids = e["input_ids"] if isinstance(e, dict) else e
            ids = np.asarray(ids, dtype=np.int64)
            if self.max_length:
                ids = ids[: self.max_length]
            if ids.size:
                seqs.append(ids)
        T = int(sum(s.size for s in seqs))
        Tp = max(self.mult, (T + self.mult - 1) // self.mult * self.mult)
        ids = np.full(Tp, self.pad_id, dtype=np.int64)
        labels = np.full(Tp, IGNORE, dtype=np.int64)
        pos = np.zeros(Tp, dtype=np.int32)
        cu = [0]
        o = 0
        for s in seqs:
            n = s.size
            ids[o:o + n] = s
            pos[o:o + n] = np.arange(n, dtype=np.int32)
            tgt = s[1:].copy()
            if self.mask_pad:
                tgt[tgt == self.pad_id] = IGNORE
            labels[o:o + n - 1] = tgt
            o += n
            cu.append(o)
        if Tp > T:
            pos[T:] = np.arange(Tp - T, dtype=np.int32)
            cu.append(Tp)
        n_valid = int((labels != IGNORE).sum())
        return {"input_ids": torch.from_numpy(ids).view(1, Tp),
                "labels": torch.from_numpy(labels).view(1, Tp),
                "pos": torch.from_numpy(pos), "cu_seqlens": tuple(cu),
                "n_valid": n_valid, "n_tokens": T, "n_padded": Tp, "n_seqs": len(seqs)}
