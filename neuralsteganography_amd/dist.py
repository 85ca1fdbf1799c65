"""Multi-GPU layer: independent streams shard across ranks.

One process per GPU (``torch.distributed``; backend ``nccl`` = RCCL on ROCm, ``gloo`` for CPU tests).
Stream s goes to rank ⌊s·world/S⌋ in contiguous slices; there is no exchange on the data path.  The only
collectives are the end-of-job reductions (bits: sum, elapsed: max) and an optional gather of token lists
to rank 0, all outside the timed coder steps.
"""

from __future__ import annotations

import os
from typing import List, Sequence, Tuple


def world_info() -> Tuple[int, int, int]:
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(total: int, world: int, rank: int) -> range:
    """Contiguous slice of ``total`` streams owned by ``rank`` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def reduce_job(bits: float, stream_steps: float, elapsed_s: float, kernel_ms: float, device=None):
    """Whole-job totals: bits and stream-steps summed over ranks, times max over ranks."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bits, stream_steps, elapsed_s, kernel_ms
    dev = device if device is not None else ("cuda" if dist.get_backend() == "nccl" else "cpu")
    s = torch.tensor([float(bits), float(stream_steps)], dtype=torch.float64, device=dev)
    m = torch.tensor([float(elapsed_s), float(kernel_ms)], dtype=torch.float64, device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return float(s[0]), float(s[1]), float(m[0]), float(m[1])


def per_rank(value: float, device=None) -> List[float]:
    """``value`` of every rank, in rank order (per-GPU times expose load imbalance from the
    variable number of tokens per stream)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(value)]
    dev = device if device is not None else ("cuda" if dist.get_backend() == "nccl" else "cpu")
    parts = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, torch.tensor([float(value)], dtype=torch.float64, device=dev))
    return [float(p[0]) for p in parts]


def gather_streams(local: Sequence, total: int) -> List:
    """Gather per-rank results (ordered by the shard of each rank) into one list of ``total`` items on
    every rank."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(local)
    world = dist.get_world_size()
    parts: List = [None] * world
    dist.all_gather_object(parts, list(local))
    out: List = [None] * total
    for r, part in enumerate(parts):
        rng = shard_range(total, world, r)
        if len(part) != len(rng):
            raise RuntimeError(f"rank {r} returned {len(part)} results for {len(rng)} streams")
        for i, item in zip(rng, part):
            out[i] = item
    return out


def encode_sharded(provider, bit_lists: Sequence[Sequence[int]], context: Sequence[int], *, quality):
    """Every rank encodes its shard with ``provider.encode_batch``; returns all token lists everywhere."""
    world, rank, _ = world_info()
    rng = shard_range(len(bit_lists), world, rank)
    local = provider.encode_batch([bit_lists[i] for i in rng], context, quality=quality) if len(rng) else []
    return gather_streams(local, len(bit_lists))


__all__ = ["world_info", "shard_range", "reduce_job", "per_rank", "gather_streams", "encode_sharded"]
