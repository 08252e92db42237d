"""Record sharding across GPUs.

Records are independent (no cross-record state in src/wal.rs:165-196 or
src/checksums.rs:20-38), so N GPUs split a batch by contiguous record ranges
and never exchange data: each shard's 4-byte results land in that shard's
slice of the output.  Fixed-size records split by count; variable-length
records split by BYTES (prefix sum of lengths cut at k * total / N), so a Zipf
tail does not leave one GPU with most of the payload.
"""
import numpy as np


def shard_fixed(n, world, rank):
    """[r0, r1) of rank's equal share of n fixed-size records."""
    per = n // world
    extra = n % world
    r0 = rank * per + min(rank, extra)
    return r0, r0 + per + (1 if rank < extra else 0)


def shard_by_bytes(lengths, world):
    """Record boundaries b[0..world] with shard k = [b[k], b[k+1]) holding ~total/world bytes."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    n = len(lengths)
    if n == 0:
        return np.zeros(world + 1, dtype=np.int64)
    csum = np.cumsum(lengths)
    total = int(csum[-1])
    cuts = [0]
    for k in range(1, world):
        target = total * k // world
        cuts.append(int(np.searchsorted(csum, target, side="right")))
    cuts.append(n)
    return np.maximum.accumulate(np.asarray(cuts, dtype=np.int64))
