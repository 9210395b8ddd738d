"""Chunk sharding across GPUs of one node.

Chunk-plan entries are independent (each decode starts from `[-1, 0]` with a fresh
context, core/asr_engine.py:1051-1060), so N GPUs run N processes, each decoding its own
share; results come back to every rank in chunk order through a host-side object gather
(no collective on the GPU data path).  The reference's own dispatch is two CPU workers
over the same chunk list (core/asr_engine.py:2250-2397).
"""
from __future__ import annotations

from typing import Callable, List, Sequence, TypeVar

R = TypeVar("R")


def lpt_partition(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of chunk indices to `world` ranks; each
    rank's list is returned in chunk order.  Deterministic (ties -> lower index / rank)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    loads = [0] * world
    parts: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (loads[k], k))
        parts[r].append(i)
        loads[r] += int(lengths[i])
    return [sorted(p) for p in parts]


def _dist():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    return dist if dist.is_available() and dist.is_initialized() else None


def decode_sharded(decode_fn: Callable[[List], List[R]], chunks: Sequence, lengths=None) -> List[R]:
    """Run `decode_fn` on this rank's LPT share of `chunks` and gather every rank's results
    in chunk order (through the group's object gather, also at world size 1).  Without an
    initialised process group this is `decode_fn(chunks)`."""
    dist = _dist()
    if dist is None:
        return list(decode_fn(list(chunks)))
    world, rank = dist.get_world_size(), dist.get_rank()
    lens = [len(c) for c in chunks] if lengths is None else list(lengths)
    mine = lpt_partition(lens, world)[rank]
    res = list(decode_fn([chunks[i] for i in mine])) if mine else []
    if len(res) != len(mine):
        raise RuntimeError("decode_fn returned %d results for %d chunks" % (len(res), len(mine)))
    gathered = [None] * world
    dist.all_gather_object(gathered, list(zip(mine, res)))
    out: List = [None] * len(chunks)
    for part in gathered:
        for i, r in part:
            out[i] = r
    return out


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (bench.py's elapsed time); identity without a group."""
    dist = _dist()
    if not dist or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
