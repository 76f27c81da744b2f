"""Data pipeline: datasets (Arrow / synthetic), tokenization, causal-LM collation, sharding.

Reference: scripts/prepare_dataset.py (glaive -> Llama-2 chat text, save_to_disk),
training/train_baseline.py:149-165 (load_from_disk, tokenize with truncation to 512, no padding),
training/train_baseline.py:195-198 (DataCollatorForLanguageModeling(mlm=False)).
"""
from .collator import CausalLMCollator, PackedCollator, shift_labels  # noqa: F401
from .loader import PrefetchLoader  # noqa: F401
from .datasets import (SyntheticTokenDataset, TokenizedDataset, build_dataset,  # noqa: F401
                       load_text_dataset)
from .sampler import ShardedSampler  # noqa: F401
from .tokenizer import ByteTokenizer, load_tokenizer  # noqa: F401
