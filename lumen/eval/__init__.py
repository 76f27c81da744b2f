"""Evaluation: held-out loss / perplexity and generation metrics.

The reference declares ``rouge-score`` and ``scikit-learn`` (requirements.txt:26-28) but never
imports them, so it has no evaluation harness.  lumen adds one so a fine-tuned adapter can be
compared against its base model:

* ``evaluate_loss``: token-weighted mean causal-LM loss and perplexity over a dataset.  It runs
  the same fused LM-head/cross-entropy kernel as training, sharded over data-parallel ranks,
  with one all-reduce of (sum of losses, token count).
* ``evaluate_generation``: greedy completions from the serving engine (paged KV,
  hipGraph decode), scored with ROUGE-1/2/L and exact match.  ROUGE is implemented here
  (``rouge_score`` is not installed).  It tokenises on whitespace and punctuation without
  stemming.

``split_llama2_chat`` turns a prepared ``<s>[INST] q [/INST] a</s>`` row
(lumen/data/prepare.py; reference scripts/prepare_dataset.py:12-25) into a (prompt, reference)
pair.
"""
from .metrics import exact_match, normalize_text, rouge_l, rouge_n, score_pairs  # noqa: F401
from .runner import evaluate_generation, evaluate_loss, split_llama2_chat  # noqa: F401
