"""Evaluation harness (lumen/eval, scripts/evaluate.py): metrics against hand-computed values,
loss/perplexity against a direct per-sequence computation, data-parallel (gloo world 2)
equivalence, and the CLI end to end on a tiny random-init model."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from lumen.eval import (evaluate_loss, exact_match, normalize_text, rouge_l, rouge_n,
                        score_pairs, split_llama2_chat)
from lumen.eval.metrics import lcs_length
from tests._dist_worker import eval_worker

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tokenisation_and_rouge_values():
    assert normalize_text("Hello, World! x=1") == ["hello", ",", "world", "!", "x", "=", "1"]
    assert lcs_length("abcbdab", "bdcaba") == 4
    # pred: the cat sat on mat (5) / ref: the cat is on the mat (6); unigram overlap 4
    p, r = "the cat sat on mat", "the cat is on the mat"
    assert rouge_n(p, r, 1) == pytest.approx(2 * (4 / 5) * (4 / 6) / (4 / 5 + 4 / 6))
    # bigrams: pred {the cat, cat sat, sat on, on mat}, ref {the cat, cat is, is on, on the,
    # the mat}: overlap 1
    assert rouge_n(p, r, 2) == pytest.approx(2 * (1 / 4) * (1 / 5) / (1 / 4 + 1 / 5))
    # LCS = the cat on mat (4)
    assert rouge_l(p, r) == pytest.approx(2 * (4 / 5) * (4 / 6) / (4 / 5 + 4 / 6))
    assert rouge_l("", "x") == 0.0 and rouge_n("a", "a", 2) == 0.0
    assert exact_match(" The  END.", "the end .") == 1.0
    s = score_pairs([("a b", "a b"), ("c", "d")])
    assert s["n"] == 2 and s["rougeL"] == pytest.approx(0.5) and s["exact_match"] == 0.5


def test_split_llama2_chat():
    q, a = split_llama2_chat("<s>[INST] How do I sort? [/INST] Use sorted(x).</s>")
    assert q == "<s>[INST] How do I sort? [/INST]" and a == "Use sorted(x)."
    assert split_llama2_chat("plain text") == ("plain text", "")


def _direct_loss(m, ds):
    tot, n = 0.0, 0
    for i in range(len(ds)):
        ids = torch.tensor(ds[i]["input_ids"])[None]
        with torch.no_grad():
            logits = m(ids).float().reshape(ids.shape[1], -1)
        lp = torch.log_softmax(logits[:-1], -1)
        tot += float(-lp.gather(1, ids[0, 1:, None]).sum())
        n += ids.shape[1] - 1
    return tot / n, n


def test_evaluate_loss_matches_direct_and_dp(tmp_path):
    from lumen.data.collator import CausalLMCollator
    from lumen.data.datasets import SyntheticTokenDataset
    from lumen.models import build_model

    m = build_model("tiny-llama", dtype=torch.float32, device=torch.device("cpu"), seed=3)
    ds = SyntheticTokenDataset(7, 24, m.config.vocab_size, seed=5, min_len=8)
    res = evaluate_loss(m, ds, CausalLMCollator(pad_id=2), batch_size=2)
    ref, n = _direct_loss(m, ds)
    assert res["eval_tokens"] == n
    assert res["eval_loss"] == pytest.approx(ref, rel=1e-5)
    assert res["perplexity"] == pytest.approx(math.exp(ref), rel=1e-5)

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(eval_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    with open(tmp_path / "eval_w2.json") as f:
        r2 = json.load(f)
    assert r2["eval_tokens"] == n           # the padded tail of the odd shard is not counted
    assert r2["eval_loss"] == pytest.approx(ref, rel=1e-5)


def test_evaluate_cli(tmp_path):
    out = tmp_path / "eval.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "evaluate.py"),
                        "--model", "tiny-llama", "--max_samples", "6", "--gen_samples", "3",
                        "--max_new_tokens", "4", "--max_length", "96", "--output", str(out)],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(out.read_text())
    assert d["samples"] == 6 and d["eval_tokens"] > 0 and math.isfinite(d["eval_loss"])
    assert d["generation"]["n"] == 3 and len(d["examples"]) == 3
