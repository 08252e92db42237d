"""Host-memory batch rate against the staging-copy thread count.

Two pageable CRC-32 batches of ~1 GiB: records packed in order (the span copy)
and the same records listed in shuffled order (the per-record gather), each
timed best of 5 per ``stage_threads`` value.  Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lsm_storage_engine_amd.device import Context  # noqa: E402


def best(fn, reps=5):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return min(ts)


def main():
    rng = np.random.default_rng(4)
    n = 1 << 19
    ln = rng.integers(64, 4033, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    total = int(off[-1]) + int(ln[-1])
    data = rng.integers(0, 256, total, dtype=np.uint8)
    perm = rng.permutation(n)
    ctx = Context(0)
    ref = ctx.crc32(data, off, ln)
    assert np.array_equal(ctx.crc32(data, off[perm], ln[perm]), ref[perm])
    res = {"payload_bytes": total, "records": n}
    for th in (1, 2, 4, 8, 16):
        ctx.set_option("stage_threads", th)
        t_span = best(lambda: ctx.crc32(data, off, ln))
        t_gather = best(lambda: ctx.crc32(data, off[perm], ln[perm]))
        res[f"span_stage{th}_GiBps"] = round(total / 2**30 / t_span, 2)
        res[f"gather_stage{th}_GiBps"] = round(total / 2**30 / t_gather, 2)
    ctx.set_option("stage_threads", 8)
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
