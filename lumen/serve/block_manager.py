"""Paged KV-cache block accounting (vLLM 0.6 block manager semantics).

The cache is ``num_blocks`` fixed-size blocks of ``block_size`` token slots per layer; a sequence
owns a block table (list of block ids) growing one block every ``block_size`` tokens.  Slot of
token t of a sequence = block_table[t // bs] * bs + t % bs.  Sizing for MI355X: the number of
blocks comes from free HBM after weights (288 GB: Llama-2-7B at 0.5 MiB/token bf16 leaves room
for ~450k cached tokens on one GPU), so preemption is rare; when it happens the scheduler frees
the youngest running sequence's blocks and recomputes it later (vLLM's recompute preemption).
"""
from __future__ import annotations

from typing import Dict, List


class NoFreeBlocks(RuntimeError):
    pass


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, watermark: float = 0.01):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.free: List[int] = list(range(num_blocks - 1, -1, -1))  # pop() -> low ids first
        self.tables: Dict[int, List[int]] = {}
        self.watermark_blocks = int(watermark * num_blocks)

    # ------------------------------------------------------------------------------------
    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    @property
    def num_free(self) -> int:
        return len(self.free)

    def can_allocate(self, n_tokens: int) -> bool:
        return self.num_free - self.blocks_needed(n_tokens) >= self.watermark_blocks

    def allocate(self, seq_id: int, n_tokens: int) -> List[int]:
        need = self.blocks_needed(n_tokens)
        if need > self.num_free:
            raise NoFreeBlocks(f"need {need} blocks, {self.num_free} free")
        tbl = self.tables.setdefault(seq_id, [])
        for _ in range(need - len(tbl)):
            tbl.append(self.free.pop())
        return tbl

    def can_append(self, seq_id: int, new_len: int) -> bool:
        have = len(self.tables.get(seq_id, []))
        return self.blocks_needed(new_len) <= have or self.num_free > 0

    def ensure(self, seq_id: int, new_len: int) -> List[int]:
        """Grow the table so it covers `new_len` tokens."""
        tbl = self.tables.setdefault(seq_id, [])
        while len(tbl) * self.block_size < new_len:
            if not self.free:
                raise NoFreeBlocks("out of KV blocks")
            tbl.append(self.free.pop())
        return tbl

    def slot(self, seq_id: int, pos: int) -> int:
        tbl = self.tables[seq_id]
        return tbl[pos // self.block_size] * self.block_size + pos % self.block_size

    def free_seq(self, seq_id: int) -> None:
        tbl = self.tables.pop(seq_id, None)
        if tbl:
            self.free.extend(reversed(tbl))

    def usage(self) -> float:
        return 1.0 - self.num_free / max(self.num_blocks, 1)
