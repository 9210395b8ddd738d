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


def gather_chunks(part: Sequence, n_all: int) -> List:
    """This rank's [(chunk index, item)] -> every rank's items of all n_all chunks, in chunk
    order (host object gather; the identity ordering without a process group).  Raises when a
    chunk is missing or delivered twice."""
    dist = _dist()
    parts = [list(part)]
    if dist is not None:
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, list(part))
    out: List = [None] * n_all
    seen = [False] * n_all
    for p in parts:
        for i, item in p:
            if seen[i]:
                raise RuntimeError(f"chunk {i} delivered twice")
            seen[i] = True
            out[i] = item
    missing = [i for i, s in enumerate(seen) if not s]
    if missing:
        raise RuntimeError(f"chunk gather lost chunks {missing[:5]}")
    return out


class RowShardedSession:
    """An ONNX-session-shaped wrapper (`run(output_names, feeds)`) that splits every call's
    batch rows over the ranks of the process group: each rank runs its contiguous share on its
    own GPU and the outputs are gathered to every rank in row order (host object gather).  All
    ranks must make the same calls with the same feeds -- true when each rank runs the same
    deterministic host logic on the same input (the config-5 restorer on the gathered
    transcript).  Rows are independent (per-sequence attention, row-wise projections), so the
    gathered outputs equal one whole-batch run (tests/test_multiproc.py, tests/test_gpu_pipe.py)."""

    def __init__(self, session):
        self.session = session

    def run(self, output_names, feeds):
        import numpy as np
        dist = _dist()
        if dist is None or dist.get_world_size() == 1:
            return self.session.run(output_names, feeds)
        world, rank = dist.get_world_size(), dist.get_rank()
        B = int(next(iter(feeds.values())).shape[0])
        lo, hi = B * rank // world, B * (rank + 1) // world
        mine = list(self.session.run(output_names, {k: v[lo:hi] for k, v in feeds.items()})) \
            if hi > lo else None
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        got = [p for p in parts if p is not None]
        return [np.concatenate([p[j] for p in got], axis=0) for j in range(len(got[0]))]


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (bench.py's elapsed time); identity without a group."""
    dist = _dist()
    if not dist or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
