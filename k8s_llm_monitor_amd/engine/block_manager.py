"""Paged KV-cache block allocator.

Uses the native allocator from ``_k8sllm_runtime`` (C++) when it is built, otherwise an
equivalent pure-Python free list.  Blocks are 16 tokens (the decode kernel's ``kBS``); a block
table row is the list of physical block ids of one sequence.
"""
from __future__ import annotations

from typing import Optional

from .sequence import Sequence


def _native():
    try:
        from ..runtime import native_runtime

        return native_runtime()
    except Exception:  # noqa: BLE001 - native runtime is optional for the allocator
        return None


class PyBlockAllocator:
    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))  # pop() hands out low ids first

    def allocate(self, n: int) -> Optional[list[int]]:
        if n > len(self._free):
            return None
        out = [self._free.pop() for _ in range(n)]
        return out

    def free(self, blocks: list[int]) -> None:
        self._free.extend(reversed(blocks))

    @property
    def num_free(self) -> int:
        return len(self._free)


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int = 16, watermark: float = 0.01,
                 use_native: bool = True):
        self.block_size = block_size
        self.num_blocks = num_blocks
        nat = _native() if use_native else None
        self.alloc = nat.BlockAllocator(num_blocks) if nat is not None else PyBlockAllocator(num_blocks)
        self.native = nat is not None
        self.watermark_blocks = max(1, int(watermark * num_blocks)) if num_blocks > 64 else 0

    def blocks_needed(self, n_tokens: int) -> int:
        return (n_tokens + self.block_size - 1) // self.block_size

    @property
    def num_free(self) -> int:
        return self.alloc.num_free

    def can_allocate(self, seq: Sequence) -> bool:
        need = self.blocks_needed(seq.num_tokens + 1)
        return self.alloc.num_free - need >= self.watermark_blocks

    def allocate(self, seq: Sequence) -> bool:
        need = self.blocks_needed(seq.num_tokens + 1)
        got = self.alloc.allocate(need)
        if got is None:
            return False
        seq.block_table = list(got)
        return True

    def ensure_slot(self, seq: Sequence) -> bool:
        """Make room for the token at position seq.num_tokens (the next decode write)."""
        need = self.blocks_needed(seq.num_tokens + 1)
        while len(seq.block_table) < need:
            got = self.alloc.allocate(1)
            if got is None:
                return False
            seq.block_table.append(got[0])
        return True

    def free(self, seq: Sequence) -> None:
        if seq.block_table:
            self.alloc.free(list(seq.block_table))
            seq.block_table = []

    def usage(self) -> float:
        return 1.0 - self.alloc.num_free / max(1, self.num_blocks)
