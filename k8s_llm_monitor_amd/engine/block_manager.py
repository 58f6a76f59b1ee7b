"""Paged KV-cache block management with prefix caching.

Blocks are 16 tokens (the kernels' block size); a block table row is the list of physical block
ids of one sequence.  The pool is reference-counted: a full block of prompt tokens is published
under a chained hash of the tokens up to its end, and a later sequence whose prompt starts with
the same tokens maps those blocks instead of recomputing them (its prefill then only runs the
remaining tokens, attending the cached prefix through the paged flash-prefill kernel).  For the
diagnostic workload every query's prompt starts with the same system preamble, and queries over
the same cluster snapshot share the whole cluster context.

Blocks whose last reference goes away stay cached (LRU) until a fresh allocation needs them.
The pool is the native ``BlockPool`` of ``_k8sllm_runtime`` (C++) when built, else an equivalent
pure-Python pool with the same hashing.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Optional

from .sequence import Sequence

_M64 = (1 << 64) - 1


def _native():
    try:
        from ..runtime import native_runtime

        return native_runtime()
    except Exception:  # noqa: BLE001 - native runtime is optional for the allocator
        return None


def _splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def py_block_hashes(tokens: list, block_size: int = 16, seed: int = 0) -> list:
    """Chained hashes of the full blocks (mirror of the native block_hashes)."""
    out = []
    h = _splitmix64(seed ^ 0x6B38C1A7D2E5F091)
    for b in range(len(tokens) // block_size):
        x = h
        for t in tokens[b * block_size:(b + 1) * block_size]:
            x = _splitmix64(x ^ (t & 0xFFFFFFFF))
        h = x or 1
        out.append(h)
    return out


class PyBlockPool:
    """Pure-Python equivalent of the native BlockPool."""

    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))
        self._ref = [0] * num_blocks
        self._hash = [0] * num_blocks
        self._lru: OrderedDict = OrderedDict()
        self._map: dict = {}
        self._stats = {"hit_blocks": 0, "queries": 0, "evictions": 0}

    def peek(self, hashes: list) -> int:
        n = 0
        for h in hashes:
            if h not in self._map:
                break
            n += 1
        return n

    def peek_idle(self, hashes: list) -> int:
        n = 0
        for h in hashes:
            b = self._map.get(h)
            if b is None:
                break
            n += self._ref[b] == 0
        return n

    def match(self, hashes: list) -> list:
        out = []
        self._stats["queries"] += 1
        for h in hashes:
            b = self._map.get(h)
            if b is None:
                break
            if self._ref[b] == 0:
                self._lru.pop(b, None)
            self._ref[b] += 1
            out.append(b)
        self._stats["hit_blocks"] += len(out)
        return out

    def allocate(self, n: int) -> Optional[list]:
        if n < 0 or n > len(self._free) + len(self._lru):
            return None
        out = []
        for _ in range(n):
            if self._free:
                b = self._free.pop()
            else:
                b, _ = self._lru.popitem(last=False)
                del self._map[self._hash[b]]
                self._hash[b] = 0
                self._stats["evictions"] += 1
            self._ref[b] = 1
            out.append(b)
        return out

    def publish(self, b: int, h: int) -> None:
        if h == 0 or self._hash[b] != 0 or h in self._map:
            return
        self._map[h] = b
        self._hash[b] = h

    def release(self, blocks: list) -> None:
        for b in reversed(blocks):
            if self._ref[b] <= 0:
                raise RuntimeError(f"double free of KV block {b}")
            self._ref[b] -= 1
            if self._ref[b] == 0:
                if self._hash[b]:
                    self._lru[b] = None
                else:
                    self._free.append(b)

    def refcount(self, b: int) -> int:
        return self._ref[b]

    def stats(self) -> dict:
        return dict(self._stats, cached_blocks=len(self._map), evictable_blocks=len(self._lru))

    @property
    def num_free(self) -> int:
        return len(self._free) + len(self._lru)

    @property
    def num_cached(self) -> int:
        return len(self._map)


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int = 16, watermark: float = 0.01,
                 use_native: bool = True, prefix_caching: bool = True):
        self.block_size = block_size
        self.num_blocks = num_blocks
        nat = _native() if use_native else None
        if nat is not None and hasattr(nat, "BlockPool"):
            self.pool = nat.BlockPool(num_blocks)
            self._hashes = lambda toks: nat.block_hashes(toks, block_size, 0)
            self.native = True
        else:
            self.pool = PyBlockPool(num_blocks)
            self._hashes = lambda toks: py_block_hashes(toks, block_size, 0)
            self.native = False
        self.prefix_caching = prefix_caching
        self.watermark_blocks = max(1, int(watermark * num_blocks)) if num_blocks > 64 else 0
        self.cached_tokens = 0  # prompt tokens served from the prefix cache (cumulative)

    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    @property
    def num_free(self) -> int:
        return self.pool.num_free

    # ------------------------------------------------------------------ prefix cache
    def _prefix_hashes(self, seq: Sequence) -> list:
        """Hashes of the full blocks that may be reused: at least one token must remain to run
        through the model (its logits give the first new token)."""
        if not self.prefix_caching:
            return []
        n = seq.num_tokens
        max_full = (n - 1) // self.block_size
        key = (n, max_full)
        if getattr(seq, "_hash_key", None) != key:
            seq._hashes = self._hashes(seq.all_ids[: max_full * self.block_size]) if max_full > 0 else []
            seq._hash_key = key
        return seq._hashes

    def cached_prefix_tokens(self, seq: Sequence) -> int:
        """Tokens of seq's prompt that the cache would serve now (no references taken)."""
        hs = self._prefix_hashes(seq)
        return self.pool.peek(hs) * self.block_size if hs else 0

    # ------------------------------------------------------------------ allocation
    def can_allocate(self, seq: Sequence) -> bool:
        """Fresh blocks needed beyond the prefix-cache hits, PLUS the hits that sit unreferenced in
        the LRU: ``match`` takes those out of the free pool too (they are counted in num_free)."""
        hs = self._prefix_hashes(seq)
        hit = self.pool.peek(hs) if hs else 0
        idle = self.pool.peek_idle(hs) if hit else 0
        need = self.blocks_needed(seq.num_tokens + 1) - hit
        return self.pool.num_free - need - idle >= self.watermark_blocks

    def allocate(self, seq: Sequence) -> bool:
        hs = self._prefix_hashes(seq)
        matched = self.pool.match(hs) if hs else []
        need = self.blocks_needed(seq.num_tokens + 1) - len(matched)
        got = self.pool.allocate(need)
        if got is None:
            if matched:
                self.pool.release(matched)
            return False
        seq.block_table = list(matched) + list(got)
        seq.num_cached = len(matched) * self.block_size
        seq.num_computed = seq.num_cached
        seq.prefilled = False
        self.cached_tokens += seq.num_cached
        return True

    def publish_computed(self, seq: Sequence, n_tokens: int) -> None:
        """Publish the full prompt blocks below position ``n_tokens`` as reusable prefixes - called
        for the tokens a prefill step is about to compute (stream order makes any later reader,
        even another sequence of the same prefill step, see them computed).  With chunked
        prefill, blocks of later chunks are published only when their chunk is scheduled."""
        hs = self._prefix_hashes(seq)
        for i in range(seq.num_cached // self.block_size, min(len(hs), n_tokens // self.block_size)):
            self.pool.publish(seq.block_table[i], hs[i])

    def ensure_slot(self, seq: Sequence) -> bool:
        """Make room for the token at position seq.num_tokens (the next decode write)."""
        need = self.blocks_needed(seq.num_tokens + 1)
        while len(seq.block_table) < need:
            got = self.pool.allocate(1)
            if got is None:
                return False
            seq.block_table.append(got[0])
        return True

    def free(self, seq: Sequence) -> None:
        if seq.block_table:
            self.pool.release(list(seq.block_table))
            seq.block_table = []
        seq.num_cached = 0
        seq.num_computed = 0
        seq.chunk = 0
        seq.prefilled = False
        seq.pending_first = 0

    def usage(self) -> float:
        return 1.0 - self.pool.num_free / max(1, self.num_blocks)

    def stats(self) -> dict:
        d = dict(self.pool.stats())
        d["prefix_cached_tokens"] = self.cached_tokens
        return d
