"""Slice-pair workloads over a FIB-SEM stack and their multi-GPU sharding.

SURVEY 8(d)/8(e): C3 = adjacent pairs (z, z+1) of a 256-slice stack; C4 = the same
on 4096 slices over 8 GPUs; C5 = gen_cross-style long-range pairs with strides
{1, 4, 16}.  Pairs are independent (the reference shards them into gzipped JSON
files of <= ppf pairs, support_scripts/gen_cross_file_list.py:26-27, one process
each); here they are cut into CONTIGUOUS chunks so the slice decoded/uploaded for
pair (z-1, z) is reused as I0 of (z, z+1), and chunks are dealt to ranks.
No data-path collective: ranks exchange only counters (RCCL/gloo all-reduce).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

Pair = Tuple[int, int]


def stack_pairs(Z: int, strides: Sequence[int] = (1,)) -> List[Pair]:
    """All (z, z + s) pairs of a Z-slice stack for each stride s (stride-major)."""
    out: List[Pair] = []
    for s in strides:
        if s <= 0:
            raise ValueError("stride must be positive")
        out.extend((z, z + s) for z in range(Z - s))
    return out


def chunks(n: int, chunk: int) -> List[Tuple[int, int]]:
    """Contiguous [start, stop) chunks covering range(n)."""
    if chunk <= 0:
        raise ValueError("chunk must be positive")
    return [(i, min(n, i + chunk)) for i in range(0, n, chunk)]


def shard(n: int, rank: int, world: int, chunk: int = 16) -> List[int]:
    """Static round-robin of contiguous chunks to ranks: rank r gets chunks
    r, r + world, ...  Every index lands on exactly one rank."""
    if not 0 <= rank < world:
        raise ValueError("bad rank")
    mine: List[int] = []
    for k, (a, b) in enumerate(chunks(n, chunk)):
        if k % world == rank:
            mine.extend(range(a, b))
    return mine


def uploads_needed(pairs: Sequence[Pair], order: Sequence[int]) -> int:
    """Slice uploads a worker does when it keeps the last two slices resident
    (the frame-reuse rule of the CLI, cli/optflow.cpp)."""
    resident: Tuple[int, int] = (-1, -1)
    n = 0
    for i in order:
        p, q = pairs[i]
        have = set(resident)
        n += (p not in have) + (q not in have)
        resident = (p, q)
    return n


class WorkQueue:
    """Work items handed out in order to whoever asks next: within a rank by a locked
    counter, across ranks by an atomic add on torch.distributed's key-value store (the
    rendezvous store: host TCP, no data-path collective)."""

    def __init__(self, n: int, store=None, key: str = "stack_q"):
        import threading
        self.n, self.store, self.key = n, store, key
        self.lock, self.next = threading.Lock(), 0

    def pop(self):
        if self.store is not None:
            i = int(self.store.add(self.key, 1)) - 1
        else:
            with self.lock:
                i, self.next = self.next, self.next + 1
        return i if i < self.n else None
