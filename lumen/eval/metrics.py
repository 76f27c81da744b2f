"""Text-overlap metrics: ROUGE-N / ROUGE-L F1 and exact match (pure Python, no rouge_score).

Tokens are lower-cased alphanumeric runs; every other non-space character is a token of its
own, so code tokens like ``(`` or ``:`` count.  ROUGE-L uses the LCS
dynamic program with two rolling rows: O(|a||b|) time and O(min) memory.
"""
from __future__ import annotations

import re
from collections import Counter
from typing import Dict, Iterable, List, Sequence, Tuple

_TOKEN = re.compile(r"[a-z0-9]+|[^\sa-z0-9]")


def normalize_text(s: str) -> List[str]:
    return _TOKEN.findall(s.lower())


def _f1(overlap: int, n_pred: int, n_ref: int) -> float:
    if overlap == 0 or n_pred == 0 or n_ref == 0:
        return 0.0
    p, r = overlap / n_pred, overlap / n_ref
    return 2 * p * r / (p + r)


def rouge_n(pred: str, ref: str, n: int = 1) -> float:
    a, b = normalize_text(pred), normalize_text(ref)
    ga = Counter(tuple(a[i:i + n]) for i in range(len(a) - n + 1))
    gb = Counter(tuple(b[i:i + n]) for i in range(len(b) - n + 1))
    overlap = sum((ga & gb).values())
    return _f1(overlap, sum(ga.values()), sum(gb.values()))


def lcs_length(a: Sequence, b: Sequence) -> int:
    if len(a) < len(b):
        a, b = b, a
    prev = [0] * (len(b) + 1)
    for x in a:
        cur = [0] * (len(b) + 1)
        for j, y in enumerate(b, start=1):
            cur[j] = prev[j - 1] + 1 if x == y else max(prev[j], cur[j - 1])
        prev = cur
    return prev[-1]


def rouge_l(pred: str, ref: str) -> float:
    a, b = normalize_text(pred), normalize_text(ref)
    return _f1(lcs_length(a, b), len(a), len(b))


def exact_match(pred: str, ref: str) -> float:
    return float(normalize_text(pred) == normalize_text(ref))


def score_pairs(pairs: Iterable[Tuple[str, str]]) -> Dict[str, float]:
    """Mean rouge1 / rouge2 / rougeL / exact_match over (prediction, reference) pairs."""
    tot = {"rouge1": 0.0, "rouge2": 0.0, "rougeL": 0.0, "exact_match": 0.0}
    n = 0
    for p, r in pairs:
        tot["rouge1"] += rouge_n(p, r, 1)
        tot["rouge2"] += rouge_n(p, r, 2)
        tot["rougeL"] += rouge_l(p, r)
        tot["exact_match"] += exact_match(p, r)
        n += 1
    return {k: v / max(n, 1) for k, v in tot.items()} | {"n": n}
