"""Index sharding of a handshake batch across ranks (one process per GPU).

Handshakes are independent (the reference runs one per call,
quantum_resistant_p2p/app/messaging.py:590, 809, 830, 1038), so N GPUs split a
batch by contiguous global index ranges and never exchange data on the hot
path.  Inputs are derived from (seed, global index), so every shard's bytes are
identical whatever the GPU count.  The only collective is the end-of-run
reduction of a few counters and the max elapsed time (RCCL over xGMI on
MI355X nodes; gloo in the CPU tests).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    first: int  # first global handshake index of this rank
    count: int  # handshakes on this rank


def weak_shard(rank: int, world: int, per_rank: int) -> Shard:
    """Weak scaling: every rank processes `per_rank` handshakes."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return Shard(rank, world, rank * per_rank, per_rank)


def strong_shard(rank: int, world: int, total: int) -> Shard:
    """Strong scaling: `total` handshakes split as evenly as possible."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return Shard(rank, world, lo, hi - lo)


DIGEST_BLOCK = 1 << 20  # global indices per shard-digest block (one library chunk)


def block_digests(rec_digests, first: int, block: int = DIGEST_BLOCK) -> dict[int, str]:
    """SHA-256 over the per-record digests (rows of a [count, 32] uint8 array, global indices
    first .. first + count) of every whole block of `block` global indices in the range:
    {block index: hex}.  Blocks are aligned to global indices, so a G-way split whose shard
    boundaries fall on block boundaries yields the same set of block digests for every G."""
    import hashlib

    import numpy as np
    d = np.ascontiguousarray(rec_digests)
    count = d.shape[0]
    if first % block or count % block:
        raise ValueError(f"shard [{first}, {first + count}) is not aligned to blocks of {block}")
    return {first // block + j: hashlib.sha256(d[j * block:(j + 1) * block].tobytes()).hexdigest()
            for j in range(count // block)}


def combine_digests(blocks: dict[int, str]) -> str:
    """One digest of the whole batch: SHA-256 over the block digests in block order."""
    import hashlib
    keys = sorted(blocks)
    if keys != list(range(len(keys))):
        raise ValueError("block digests do not tile the batch")
    return hashlib.sha256(b"".join(bytes.fromhex(blocks[k]) for k in keys)).hexdigest()


def gather_digests(blocks: dict[int, str]) -> dict[int, str]:
    """Union of every rank's block digests (identity when not distributed)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(blocks)
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, blocks)
    out: dict[int, str] = {}
    for p in parts:
        out.update(p)
    return out


def reduce_run(elapsed_s: float, counters: list[int], device=None) -> tuple[float, list[int]]:
    """max(elapsed) and sum(counters) over all ranks (identity when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed_s, list(counters)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    c = torch.tensor(list(counters), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(x) for x in c.tolist()]
