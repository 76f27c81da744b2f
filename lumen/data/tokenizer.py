"""Tokenizer loading (offline).

Reference: ``AutoTokenizer.from_pretrained(model_name)``, pad := eos when missing
(training/train_baseline.py:115-117).  The GPU boxes have no network, so: a local directory with
``tokenizer.json`` is loaded through the `tokenizers` library (installed); otherwise a
deterministic byte-level tokenizer stands in (ids 3..258 = bytes, 0 pad/unk, 1 bos, 2 eos), which
keeps the whole pipeline runnable on synthetic / local text.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional


class ByteTokenizer:
    pad_token_id = 0
    bos_token_id = 1
    eos_token_id = 2
    offset = 3

    def __init__(self, vocab_size: int = 32000, add_bos: bool = True):
        self.vocab_size = vocab_size
        self.add_bos = add_bos
        self.pad_token_id = self.eos_token_id  # reference: pad = eos

    def encode(self, text: str, add_special_tokens: bool = True) -> List[int]:
        ids = [b + self.offset for b in text.encode("utf-8")]
        return ([self.bos_token_id] if (self.add_bos and add_special_tokens) else []) + ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        bs = bytes(i - self.offset for i in ids if self.offset <= i < self.offset + 256)
        return bs.decode("utf-8", errors="replace")

    def __call__(self, texts, truncation=True, max_length=None, padding=False):
        if isinstance(texts, str):
            texts = [texts]
        out = []
        for t in texts:
            ids = self.encode(t)
            if truncation and max_length:
                ids = ids[:max_length]
            out.append(ids)
        return {"input_ids": out}

    def save_pretrained(self, path: str):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "lumen_tokenizer.json"), "w") as f:
            json.dump({"type": "byte", "vocab_size": self.vocab_size, "add_bos": self.add_bos}, f)


class HFTokenizer:
    """Thin wrapper over `tokenizers.Tokenizer` loaded from a local tokenizer.json."""

    def __init__(self, path: str):
        from tokenizers import Tokenizer

        self.path = path
        self.tok = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
        cfg = {}
        tc = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(tc):
            with open(tc) as f:
                cfg = json.load(f)

        def tid(name, default):
            t = cfg.get(name)
            if isinstance(t, dict):
                t = t.get("content")
            if t is None:
                return default
            i = self.tok.token_to_id(t)
            return default if i is None else i

        self.bos_token_id = tid("bos_token", 1)
        self.eos_token_id = tid("eos_token", 2)
        pad = tid("pad_token", None)
        self.pad_token_id = pad if pad is not None else self.eos_token_id
        self.vocab_size = self.tok.get_vocab_size()

    def encode(self, text: str, add_special_tokens: bool = True) -> List[int]:
        return self.tok.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        return self.tok.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def __call__(self, texts, truncation=True, max_length=None, padding=False):
        if isinstance(texts, str):
            texts = [texts]
        out = []
        for t in texts:
            ids = self.encode(t)
            if truncation and max_length:
                ids = ids[:max_length]
            out.append(ids)
        return {"input_ids": out}

    def save_pretrained(self, path: str):
        import shutil

        os.makedirs(path, exist_ok=True)
        for fn in ("tokenizer.json", "tokenizer_config.json", "special_tokens_map.json",
                   "tokenizer.model"):
            src = os.path.join(self.path, fn)
            if os.path.exists(src):
                shutil.copy(src, os.path.join(path, fn))


def load_tokenizer(name_or_path: Optional[str], vocab_size: int = 32000):
    if name_or_path and os.path.isdir(name_or_path) and \
            os.path.exists(os.path.join(name_or_path, "tokenizer.json")):
        return HFTokenizer(name_or_path)
    return ByteTokenizer(vocab_size)
