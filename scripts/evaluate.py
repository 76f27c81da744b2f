#!/usr/bin/env python
"""Evaluate a base model or a fine-tuned LoRA adapter: held-out loss/perplexity and greedy
generation ROUGE / exact match (lumen/eval).

    python scripts/evaluate.py --model meta-llama/Llama-2-7b-hf \
        --adapter checkpoints/zero3_8gpu/final --dataset_path ./data/glaive_code_2k \
        --max_samples 256 --max_new_tokens 128 --output results/eval.json

``--dataset_path`` is a prepared Arrow dir / .jsonl / .json / .txt (``text`` rows in the Llama-2
chat format); without it, or with ``--synthetic``, the evaluation runs on the offline synthetic
Q&A rows from scripts/prepare_dataset.py.  ``--skip_generation`` / ``--skip_loss`` select one
half.  With several processes (``python -m lumen.launch --nproc_per_node N``) the loss pass is
data-parallel; generation runs on rank 0.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(argv=None):
    p = argparse.ArgumentParser(description="lumen evaluation: perplexity + ROUGE")
    p.add_argument("--model", required=True)
    p.add_argument("--adapter", default=None)
    p.add_argument("--dataset_path", default=None)
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--max_samples", type=int, default=256)
    p.add_argument("--max_length", type=int, default=512)
    p.add_argument("--batch_size", type=int, default=8)
    p.add_argument("--max_new_tokens", type=int, default=128)
    p.add_argument("--gen_samples", type=int, default=64)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    p.add_argument("--skip_loss", action="store_true")
    p.add_argument("--skip_generation", action="store_true")
    p.add_argument("--output", default=None)
    a = p.parse_args(argv)

    import torch
    import torch.distributed as dist

    from lumen.data.collator import CausalLMCollator
    from lumen.data.datasets import TokenizedDataset, load_text_dataset
    from lumen.data.prepare import format_conversation_for_llama2, synthetic_rows
    from lumen.data.tokenizer import load_tokenizer
    from lumen.eval import evaluate_generation, evaluate_loss, split_llama2_chat
    from lumen.models import build_model

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    on_gpu = torch.cuda.is_available()
    if on_gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    if world > 1:
        dist.init_process_group("nccl" if on_gpu else "gloo")
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    if not on_gpu:
        dt = torch.float32

    if a.dataset_path and not a.synthetic and os.path.exists(a.dataset_path):
        texts = load_text_dataset(a.dataset_path)
    else:
        texts = [format_conversation_for_llama2(r)["text"] for r in synthetic_rows(a.max_samples)]
    texts = texts[: a.max_samples]

    model = build_model(a.model, dtype=dt, device=dev)
    tok = load_tokenizer(a.adapter if a.adapter and os.path.isfile(
        os.path.join(a.adapter, "tokenizer_config.json")) else a.model, model.config.vocab_size)
    if a.adapter:
        from lumen.lora import load_adapter

        load_adapter(model, a.adapter)
    out = {"model": a.model, "adapter": a.adapter, "samples": len(texts)}

    if not a.skip_loss:
        enc = tok(texts, truncation=True, max_length=a.max_length, padding=False)
        ds = TokenizedDataset(enc["input_ids"])
        pad = tok.pad_token_id if getattr(tok, "pad_token_id", None) is not None else tok.eos_token_id
        coll = CausalLMCollator(pad_id=pad, max_length=a.max_length)
        out.update(evaluate_loss(model, ds, coll, a.batch_size, dev, rank, world))

    if not a.skip_generation and rank == 0:
        from lumen.lora import merge_lora
        from lumen.serve.engine import EngineConfig, LLMEngine

        pairs = [split_llama2_chat(t) for t in texts[: a.gen_samples]]
        pairs = [(q, r) for q, r in pairs if r]
        if pairs:
            merge_lora(model)  # serving runs on merged weights (adapters folded in)
            max_len = a.max_length + a.max_new_tokens
            eng = LLMEngine(EngineConfig(model=a.model, dtype=a.dtype, max_model_len=max_len,
                                         max_num_seqs=min(64, len(pairs)),
                                         device=str(dev), use_graphs=on_gpu),
                            model=model, tokenizer=tok)
            # prompts are truncated from the left so the instruction tail survives
            prompts = [tok.encode(q)[-a.max_length:] for q, _ in pairs]
            res = evaluate_generation(eng, prompts, [r for _, r in pairs], a.max_new_tokens)
            out["generation"] = res["metrics"]
            out["examples"] = [{"reference": r[:200], "prediction": pr[:200]}
                               for (_, r), pr in zip(pairs[:4], res["predictions"][:4])]

    if rank == 0:
        print(json.dumps({k: v for k, v in out.items() if k != "examples"}))
        if a.output:
            os.makedirs(os.path.dirname(os.path.abspath(a.output)), exist_ok=True)
            with open(a.output, "w") as f:
                json.dump(out, f, indent=2)
    if world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
