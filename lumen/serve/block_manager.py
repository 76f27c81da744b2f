"""Paged KV-cache block accounting (vLLM 0.6 block manager semantics).

The cache is ``num_blocks`` fixed-size blocks of ``block_size`` token slots per layer; a sequence
owns a block table (list of block ids) growing one block every ``block_size`` tokens.  Slot of
token t of a sequence = block_table[t // bs] * bs + t % bs.  Sizing for MI355X: the number of
blocks comes from free HBM after weights (288 GB: Llama-2-7B at 0.5 MiB/token bf16 leaves room
for ~450k cached tokens on one GPU), so preemption is rare; when it happens the scheduler frees
the youngest running sequence's blocks and recomputes it later (vLLM's recompute preemption).

Automatic prefix caching (``prefix_caching=True``; vLLM's ``--enable-prefix-caching``, off by
default there as here).  A FULL block is named by a 128-bit digest of (previous block's digest,
adapter slot, its token ids), so equal digests mean equal token prefixes and equal K/V.  Blocks
are reference-counted:

* admission looks the prompt's full blocks up in order and shares the hits (at most
  ``(len - 1) // bs`` of them: at least one token is computed, its logits give the first sample,
  and every write of the sequence lands in a block of its own -- shared blocks are read-only);
* a block is named (published) once the step that writes its K/V is launched: prompt blocks at
  their prefill's launch (later steps of the same burst already hit them), generated tokens'
  blocks when the sequence finishes (a multi-turn conversation's next prompt hits its previous
  turn);
* a block whose count drops to zero keeps its digest and parks in an LRU list; allocation takes
  never-used / unnamed blocks first, then evicts the least recently released named one.

With 288 GB of HBM the parked blocks are a large cache (hundreds of thousands of tokens for a
7B model) that costs nothing until allocation needs the space.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence as Seq

import numpy as np


class NoFreeBlocks(RuntimeError):
    pass


def block_digest(parent: bytes, lora: int, tokens: Seq[int]) -> bytes:
    """Name of a full block: its token ids chained to the previous block's name."""
    h = hashlib.blake2b(parent, digest_size=16)
    h.update(int(lora).to_bytes(4, "little", signed=True))
    h.update(np.asarray(tokens, dtype=np.int64).tobytes())
    return h.digest()


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, watermark: float = 0.01,
                 prefix_caching: bool = False):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.free: List[int] = list(range(num_blocks - 1, -1, -1))  # pop() -> low ids first
        self.tables: Dict[int, List[int]] = {}
        self.watermark_blocks = int(watermark * num_blocks)
        self.prefix_caching = prefix_caching
        # prefix cache state (empty unless prefix_caching)
        self.ref: Dict[int, int] = {}                    # block -> sequences holding it
        self.cached: Dict[bytes, int] = {}               # digest -> block
        self.name: Dict[int, bytes] = {}                 # block -> digest
        self.parked: "OrderedDict[int, None]" = OrderedDict()  # named, unreferenced (LRU first)
        self.chains: Dict[Optional[int], List[bytes]] = {}   # seq -> names of its full blocks
        self.stale: set = set()  # running sequences whose K/V predate a reset: never published
        self.hit_tokens = 0
        self.query_tokens = 0

    # ------------------------------------------------------------------------------------
    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    @property
    def num_free(self) -> int:
        return len(self.free) + len(self.parked)

    def can_allocate(self, n_tokens: int) -> bool:
        return self.num_free - self.blocks_needed(n_tokens) >= self.watermark_blocks

    def _take(self) -> int:
        """One block for a new write: an unnamed free block, else evict the LRU parked one."""
        if self.free:
            b = self.free.pop()
        elif self.parked:
            b, _ = self.parked.popitem(last=False)
            del self.cached[self.name.pop(b)]
        else:
            raise NoFreeBlocks("out of KV blocks")
        if self.prefix_caching:
            self.ref[b] = 1
        return b

    def _digests(self, ids: Seq[int], n_blocks: int, lora: int,
                 seq_id: Optional[int] = None) -> List[bytes]:
        """Names of the first ``n_blocks`` full blocks of ``ids`` (memoised per sequence: a
        chunked prompt's blocks are named once)."""
        bs = self.block_size
        out = self.chains.setdefault(seq_id, []) if seq_id is not None else []
        while len(out) < n_blocks:
            j = len(out)
            out.append(block_digest(out[-1] if out else b"", lora, ids[j * bs:(j + 1) * bs]))
        return out[:n_blocks]

    def publish(self, seq_id: int, token_ids: Seq[int], n_computed: int, lora: int = 0) -> None:
        """Name the sequence's full blocks among its first ``n_computed`` tokens (their K/V are
        written by steps already launched, so any later step may read them).  A block whose
        content is already cached under another id stays unnamed."""
        tbl = self.tables.get(seq_id)
        if not self.prefix_caching or not tbl or seq_id in self.stale:
            return
        nfull = min(n_computed, len(token_ids), len(tbl) * self.block_size) // self.block_size
        for b, d in zip(tbl[:nfull], self._digests(token_ids, nfull, lora, seq_id)):
            if b not in self.name and d not in self.cached:
                self.cached[d] = b
                self.name[b] = d

    def allocate(self, seq_id: int, n_tokens: int, token_ids: Optional[Seq[int]] = None,
                 lora: int = 0) -> int:
        """Table covering ``n_tokens`` slots for a new sequence.  With prefix caching and the
        sequence's ``token_ids``, the leading full blocks found in the cache are shared; returns
        the number of tokens whose K/V are thereby already cached (0 without prefix caching)."""
        need = self.blocks_needed(n_tokens)
        tbl = self.tables.setdefault(seq_id, [])
        hits: List[int] = []
        if self.prefix_caching and token_ids is not None and not tbl:
            for d in self._digests(token_ids, (len(token_ids) - 1) // self.block_size, lora,
                                   seq_id):
                b = self.cached.get(d)
                if b is None:
                    break
                hits.append(b)
        # blocks still to take; parked hits leave the parked pool without being taken
        parked_hits = sum(1 for b in hits if b in self.parked)
        if need - len(tbl) - len(hits) > self.num_free - parked_hits:
            raise NoFreeBlocks(f"need {need} blocks, {self.num_free} free")
        if self.prefix_caching and token_ids is not None and not tbl:
            self.query_tokens += len(token_ids)
            self.hit_tokens += len(hits) * self.block_size
        for b in hits:
            self.parked.pop(b, None)
            self.ref[b] = self.ref.get(b, 0) + 1
            tbl.append(b)
        for _ in range(need - len(tbl)):
            tbl.append(self._take())
        return len(hits) * self.block_size

    def can_append(self, seq_id: int, new_len: int) -> bool:
        have = len(self.tables.get(seq_id, []))
        return self.blocks_needed(new_len) <= have or self.num_free > 0

    def ensure(self, seq_id: int, new_len: int) -> List[int]:
        """Grow the table so it covers `new_len` tokens."""
        tbl = self.tables.setdefault(seq_id, [])
        while len(tbl) * self.block_size < new_len:
            tbl.append(self._take())
        return tbl

    def slot(self, seq_id: int, pos: int) -> int:
        tbl = self.tables[seq_id]
        return tbl[pos // self.block_size] * self.block_size + pos % self.block_size

    def free_seq(self, seq_id: int, token_ids: Optional[Seq[int]] = None, n_computed: int = 0,
                 lora: int = 0) -> None:
        """Release a sequence's blocks.  With prefix caching, ``token_ids`` / ``n_computed``
        (tokens whose K/V its launched steps wrote) publish its full blocks first; a block
        whose content is already cached under another id is simply released."""
        if not self.prefix_caching:
            tbl = self.tables.pop(seq_id, None)
            if tbl:
                self.free.extend(reversed(tbl))
            return
        if token_ids is not None:
            self.publish(seq_id, token_ids, n_computed, lora)
        self.stale.discard(seq_id)
        self.chains.pop(seq_id, None)
        tbl = self.tables.pop(seq_id, None)
        if not tbl:
            return
        for b in reversed(tbl):
            r = self.ref.get(b, 1) - 1
            if r > 0:
                self.ref[b] = r
                continue
            self.ref.pop(b, None)
            if b in self.name:
                self.parked[b] = None        # most recently released last
            else:
                self.free.append(b)

    def reset_prefix_cache(self) -> None:
        """Forget every block's name (the cache's content is no longer trusted, e.g. after the
        weights changed): parked blocks become free; blocks in use are freed unnamed, and the
        sequences holding them never publish (their K/V were computed before the reset)."""
        self.free.extend(reversed(list(self.parked)))
        self.parked.clear()
        self.cached.clear()
        self.name.clear()
        self.chains.clear()
        self.stale.update(self.tables)

    def usage(self) -> float:
        return 1.0 - self.num_free / max(self.num_blocks, 1)

    @property
    def hit_rate(self) -> float:
        return self.hit_tokens / self.query_tokens if self.query_tokens else 0.0
