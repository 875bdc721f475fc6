"""Sample sharding for multi-GPU runs.

Each rank owns a contiguous shard of the trajectory batch; the device library
all-reduces the un-normalised P-sized partial sum once per FVP over RCCL and
divides by the GLOBAL sample count, so every rank runs an identical CG.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of samples owned by `rank`; sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world %d/%d" % (rank, world))
    return n * rank // world, n * (rank + 1) // world
