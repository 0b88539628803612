"""Multi-GPU sharding of checksum batches: one process per GPU, no collective on the data path.

Records are independent (every smoltcp `Repr::parse` / `Repr::emit` checksums one packet), so a
batch splits into contiguous record ranges, one per rank, and each rank runs the batched engine
on its own range in its own HBM.  The only collectives are for reporting: a barrier around the
timed region and a max-reduction of the elapsed time (`bench.py`).  `torch.distributed` is used
with RCCL (`"nccl"`) on GPUs and `gloo` in the CPU tests.

Two ways to use it:

* weak scaling (`bench.py`): every rank synthesises its own batch from `rank_seed(base, rank)`;
* partitioning one global batch (a capture, a ring dump): `shard_range` / `shard_fixed` /
  `shard_records` give rank r its record range, the byte range of the global buffer it must copy
  into its HBM, and the batch geometry relative to that copy (descriptor offsets rebased).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np


def dist_env():
    """(world, rank, local_rank) from the torch.distributed.run environment (1, 0, 0 without)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n: int, rank: int, world: int):
    """Balanced contiguous record range [lo, hi) of rank `rank` out of `world` (sizes differ by
    at most one record; the first n % world ranks take the extra record)."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError(f"bad shard ({rank} of {world}, n={n})")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def rank_seed(base: int, rank: int) -> int:
    """Seed of rank `rank`'s synthetic batch (distinct batches per rank in weak scaling)."""
    return (int(base) + 1000 * int(rank)) & (2**64 - 1)


@dataclass
class Shard:
    """Rank-local part of a global batch.

    `byte_lo`/`byte_hi`: the slice of the global buffer the rank copies into its HBM.  The
    geometry (`n`, `stride`, `length`, or `desc` with offsets relative to `byte_lo`) describes
    the records inside that copy."""

    lo: int
    hi: int
    byte_lo: int
    byte_hi: int
    stride: int = 0
    length: int = 0
    desc: Optional[np.ndarray] = None  # host smol_csum_desc_t array (engine.DESC_DTYPE), rebased

    @property
    def n(self) -> int:
        return self.hi - self.lo


def shard_fixed(n: int, stride: int, length: int, rank: int, world: int) -> Shard:
    """Fixed-stride batch: record i at i*stride, `length` bytes."""
    lo, hi = shard_range(n, rank, world)
    if hi == lo:
        return Shard(lo, hi, 0, 0, stride, length)
    return Shard(lo, hi, lo * stride, (hi - 1) * stride + length, stride, length)


def shard_records(desc: np.ndarray, rank: int, world: int) -> Shard:
    """Descriptor batch (host `engine.DESC_DTYPE` array, any offsets): the rank's descriptors,
    rebased to the start of the smallest byte range that holds all of its records."""
    lo, hi = shard_range(len(desc), rank, world)
    d = desc[lo:hi].copy()
    if hi == lo:
        return Shard(lo, hi, 0, 0, desc=d)
    off = d["offset"].astype(np.uint64)
    end = off + d["len"].astype(np.uint64)
    b0, b1 = int(off.min()), int(end.max())
    d["offset"] = off - np.uint64(b0)
    return Shard(lo, hi, b0, b1, desc=d)


def max_over_ranks(value: float, device=None) -> float:
    """Max of a float over all ranks (identity when torch.distributed is not initialised).  With
    RCCL the tensor must live on the rank's GPU; with gloo on the CPU."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(bytes_per_rank_per_step: int, world: int, steps: int, elapsed_s: float) -> float:
    """Whole-job GiB/s: the bytes all ranks processed over the max-over-ranks elapsed time."""
    return bytes_per_rank_per_step * world * steps / elapsed_s / float(1 << 30)
