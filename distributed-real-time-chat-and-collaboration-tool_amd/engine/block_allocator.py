"""Block allocator front-end: the native C++ allocator (csrc/runtime/
block_allocator.h) with a pure-Python twin used only if ``_native`` has not
been built (e.g. a source checkout before ``python -m drtc_amd._build``)."""
from __future__ import annotations

import importlib


class PyBlockAllocator:
    def __init__(self, num_blocks: int, reserved: int = 0):
        if num_blocks <= reserved:
            raise ValueError("num_blocks must exceed reserved")
        self.num_blocks = num_blocks
        self._reserved = reserved
        self._free = list(range(num_blocks - 1, reserved - 1, -1))
        self._ref = [0] * num_blocks

    @property
    def num_free(self) -> int:
        return len(self._free)

    @property
    def num_used(self) -> int:
        return self.num_blocks - self._reserved - len(self._free)

    def can_allocate(self, n: int) -> bool:
        return n <= len(self._free)

    def allocate(self, n: int) -> list[int]:
        if n > len(self._free):
            raise RuntimeError("BlockAllocator: out of KV-cache blocks")
        out = [self._free.pop() for _ in range(n)]
        for b in out:
            self._ref[b] = 1
        return out

    def allocate_one(self) -> int:
        return self.allocate(1)[0]

    def incref(self, blocks) -> None:
        for b in blocks:
            if self._ref[b] <= 0:
                raise RuntimeError("BlockAllocator: incref of a free block")
            self._ref[b] += 1

    def free(self, blocks) -> None:
        for b in blocks:
            if not (self._reserved <= b < self.num_blocks):
                raise IndexError("BlockAllocator: block id out of range")
            if self._ref[b] <= 0:
                raise RuntimeError("BlockAllocator: double free")
            self._ref[b] -= 1
            if self._ref[b] == 0:
                self._free.append(b)

    def refcount(self, b: int) -> int:
        return self._ref[b]


def _native_cls():
    try:
        pkg = __name__.rsplit(".", 2)[0]
        return importlib.import_module(pkg + "._native").BlockAllocator
    except ImportError:
        return None


def BlockAllocator(num_blocks: int, reserved: int = 0):
    cls = _native_cls()
    if cls is None:
        return PyBlockAllocator(num_blocks, reserved)
    return cls(num_blocks, reserved)
