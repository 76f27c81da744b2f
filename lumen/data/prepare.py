"""Instruction-dataset preparation (reference scripts/prepare_dataset.py:12-121).

The reference downloads ``glaiveai/glaive-code-assistant`` from the HF Hub, formats every
(question, answer) pair as a Llama-2 chat string ``"<s>[INST] {q} [/INST] {a}</s>"``
(:12-25) and writes an Arrow dir with a single ``text`` column named ``glaive_code_full`` or
``glaive_code_{N//1000}k`` (:86-92).  lumen keeps that on-disk contract but never needs the
network: the source can be a local JSON / JSONL / parquet / CSV file or an Arrow dir with
``question``/``answer`` columns (the glaive schema), the HF Hub when it is reachable, or a
deterministic synthetic Q&A corpus (``source="synthetic"``) so the whole pipeline runs offline.
"""
from __future__ import annotations

import json
import os
import random
from pathlib import Path
from typing import Dict, Iterable, List, Optional

GLAIVE_HUB_ID = "glaiveai/glaive-code-assistant"


def format_conversation_for_llama2(example: Dict) -> Dict:
    """Llama-2 chat template of one glaive row (reference scripts/prepare_dataset.py:12-25).

    The literal ``<s>``/``</s>`` are kept in the text for byte-compatibility with datasets the
    reference produced (the tokenizer adds a second BOS)."""
    q = str(example.get("question", "")).strip()
    a = str(example.get("answer", "")).strip()
    return {"text": f"<s>[INST] {q} [/INST] {a}</s>"}


def dataset_dir_name(num_samples: Optional[int]) -> str:
    """``glaive_code_full`` or ``glaive_code_{N//1000}k`` (reference :86-87)."""
    return "glaive_code_full" if not num_samples else f"glaive_code_{num_samples // 1000}k"


_TOPICS = ["sort a list", "reverse a string", "parse JSON", "read a CSV file", "compute a mean",
           "merge two dicts", "find duplicates", "binary search", "count words",
           "flatten a nested list", "format a date", "validate an email", "memoize a function",
           "open a socket", "compute a factorial", "transpose a matrix"]
_LANGS = ["Python", "C++", "JavaScript", "Rust", "Go", "Java", "Bash", "SQL"]


def synthetic_rows(n: int, seed: int = 42) -> List[Dict]:
    """Deterministic code-assistant-like Q&A rows (offline stand-in for the glaive corpus)."""
    rng = random.Random(seed)
    rows = []
    for i in range(n):
        topic, lang = rng.choice(_TOPICS), rng.choice(_LANGS)
        name = topic.replace(" ", "_").replace("-", "_")
        body = "\n".join(f"    step_{j} = step_{j - 1} if {j} else arg" for j in range(rng.randint(2, 12)))
        q = f"How can I {topic} in {lang}? (example {i})"
        a = (f"Here is one way to {topic} in {lang}:\n\n```\ndef {name}(arg):\n{body}\n"
             f"    return step_{0}\n```\nThis runs in linear time for typical inputs.")
        rows.append({"question": q, "answer": a})
    return rows


def _read_local(path: str) -> List[Dict]:
    if os.path.isdir(path):
        from datasets import load_from_disk

        ds = load_from_disk(path)
        if hasattr(ds, "keys") and "train" in ds:
            ds = ds["train"]
        return [dict(r) for r in ds]
    if path.endswith(".jsonl"):
        with open(path) as f:
            return [json.loads(l) for l in f if l.strip()]
    if path.endswith(".json"):
        with open(path) as f:
            data = json.load(f)
        return data if isinstance(data, list) else data.get("data", data.get("train", []))
    if path.endswith(".parquet"):
        import pyarrow.parquet as pq

        return pq.read_table(path).to_pylist()
    if path.endswith(".csv"):
        import csv

        with open(path, newline="") as f:
            return list(csv.DictReader(f))
    raise ValueError(f"unsupported source file: {path}")


def load_source(source: str, num_samples: Optional[int], seed: int = 42) -> List[Dict]:
    """``synthetic`` | ``hub`` | a local path (see module docstring)."""
    if source == "synthetic":
        return synthetic_rows(num_samples or 2000, seed)
    if source == "hub":
        from datasets import load_dataset  # needs network or a warm HF cache

        ds = load_dataset(GLAIVE_HUB_ID, split="train")
        if num_samples:
            ds = ds.select(range(min(num_samples, len(ds))))
        return [dict(r) for r in ds]
    rows = _read_local(source)
    return rows[:num_samples] if num_samples else rows


def prepare_dataset(output_dir: str = "./data", num_samples: Optional[int] = None,
                    source: str = "synthetic", seed: int = 42) -> str:
    """Format + save as an Arrow dir with one ``text`` column; returns the saved path."""
    from datasets import Dataset

    rows = load_source(source, num_samples, seed)
    texts = [format_conversation_for_llama2(r)["text"] for r in rows
             if "question" in r or "answer" in r]
    if not texts:  # already formatted rows
        texts = [r["text"] for r in rows if "text" in r]
    out = Path(output_dir) / dataset_dir_name(num_samples)
    out.parent.mkdir(parents=True, exist_ok=True)
    Dataset.from_dict({"text": texts}).save_to_disk(str(out))
    return str(out)


def dir_size_mb(path: str) -> float:
    total = 0
    for root, _, files in os.walk(path):
        for f in files:
            total += os.path.getsize(os.path.join(root, f))
    return total / 1e6


def iter_texts(rows: Iterable[Dict]):
    for r in rows:
        yield format_conversation_for_llama2(r)["text"]
