"""Datasets: Arrow text datasets (the reference's on-disk format) and synthetic token data.

Reference on-disk layout: ``datasets`` Arrow dir with one ``text`` column
(scripts/prepare_dataset.py:25,92), loaded by ``load_from_disk`` and tokenized with truncation
to 512 and no padding (training/train_baseline.py:149-165).  Benchmarks use
``SyntheticTokenDataset`` (random token ids of a fixed length: no network on the GPU boxes).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch


class SyntheticTokenDataset:
    """`n` sequences of `seq_len` uniformly random token ids in [3, vocab) (ids 0-2 special)."""

    def __init__(self, n: int, seq_len: int, vocab_size: int, seed: int = 1234,
                 min_len: Optional[int] = None):
        self.n, self.seq_len, self.vocab = n, seq_len, vocab_size
        self.seed = seed
        self.min_len = min_len

    def __len__(self):
        return self.n

    def _len(self, g) -> int:
        if self.min_len is not None and self.min_len < self.seq_len:
            return int(torch.randint(self.min_len, self.seq_len + 1, (1,), generator=g))
        return self.seq_len

    def length(self, i) -> int:
        """Row length without generating the row (token-budget batch planning)."""
        return self._len(torch.Generator().manual_seed(self.seed * 1_000_003 + i))

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        ids = torch.randint(3, self.vocab, (self._len(g),), generator=g)
        return {"input_ids": ids.tolist()}


class TokenizedDataset:
    def __init__(self, rows: List[List[int]]):
        self.rows = rows

    def __len__(self):
        return len(self.rows)

    def __getitem__(self, i):
        return {"input_ids": self.rows[i]}

    def length(self, i) -> int:
        return len(self.rows[i])


def load_text_dataset(path: str):
    """Arrow dir (datasets.save_to_disk), .jsonl / .json (list of {"text"}), or .txt lines."""
    if os.path.isdir(path):
        from datasets import load_from_disk

        ds = load_from_disk(path)
        if hasattr(ds, "keys") and "train" in ds:
            ds = ds["train"]
        return [r["text"] for r in ds]
    if path.endswith(".jsonl"):
        import json

        with open(path) as f:
            return [json.loads(l)["text"] for l in f if l.strip()]
    if path.endswith(".json"):
        import json

        with open(path) as f:
            return [r["text"] for r in json.load(f)]
    with open(path) as f:
        return [l.rstrip("\n") for l in f if l.strip()]


def build_dataset(dataset_path: Optional[str], tokenizer, max_length: int, synthetic: bool,
                  synthetic_samples: int, vocab_size: int, seed: int = 1234,
                  synthetic_min_len: Optional[int] = None):
    if synthetic or not dataset_path or not os.path.exists(dataset_path):
        return SyntheticTokenDataset(synthetic_samples, max_length, vocab_size, seed,
                                     synthetic_min_len)
    texts = load_text_dataset(dataset_path)
    enc = tokenizer(texts, truncation=True, max_length=max_length, padding=False)
    return TokenizedDataset(enc["input_ids"])
