#!/usr/bin/env python3
"""SHA-256 kernel rate by message size class (diagnostic for DESIGN.md 8).

Config 3's Zipf lengths split into block-count classes.  For each class, the
messages are packed into their own device buffer and hashed with one
lsmck_sha256_batch (device pointers, length-ordered dispatch), timed with HIP
events.  The rate is compression blocks per second, next to the same rate for
fixed 4 KiB messages (config 2's shape).

  python3 tools/sha_buckets.py [--records N]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch  # first: liblsmck binds to torch's HIP runtime

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lsm_storage_engine_amd.device import Context, gen_zipf_lengths  # noqa: E402

CLASSES = [(2, 2), (3, 3), (4, 8), (9, 32), (33, 128), (129, 2048)]


def timed(ctx, stream, fn, reps=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    ctx.sync(stream.cuda_stream)
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--presorted", action="store_true",
                    help="pack each class's messages in decreasing block-count order, so a wave's lanes read "
                         "neighbouring messages (locality / TLB-reach diagnostic)")
    a = ap.parse_args()
    ctx = Context(0)
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    ln_all = gen_zipf_lengths(0x5EED0003, a.records)
    nb_all = (ln_all.astype(np.int64) + 72) >> 6
    res = {"records": a.records, "classes": []}
    for lo, hi in CLASSES:
        sel = (nb_all >= lo) & (nb_all <= hi)
        ln = ln_all[sel].astype(np.uint32)
        if a.presorted:
            ln = ln[np.argsort(-((ln.astype(np.int64) + 72) >> 6), kind="stable")]
        n = len(ln)
        if n < 64:
            continue
        off = np.zeros(n, dtype=np.uint64)
        np.cumsum(ln[:-1].astype(np.uint64), out=off[1:])
        total = int(off[-1]) + int(ln[-1])
        d = ctx.alloc(total + 64)
        ctx.gen_stream(d.ptr, 0x5EED0003, 0, total, sp)
        d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(32 * n)
        d_o.upload(off)
        d_l.upload(ln)
        ms = timed(ctx, stream, lambda: ctx.sha256_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr, sp))
        blocks = int(nb_all[sel].sum())
        res["classes"].append({"blocks_per_msg": [lo, hi], "messages": n, "bytes": total, "ms": round(ms, 3),
                               "Gblocks_per_s": round(blocks / ms / 1e6, 3)})
        print(res["classes"][-1], flush=True)
        for b in (d, d_o, d_l, out):
            b.free()
    n = 1 << 22
    d, out = ctx.alloc(n * 4096), ctx.alloc(32 * n)
    ctx.gen_stream(d.ptr, 0x5EED0002, 0, n * 4096, sp)
    ms = timed(ctx, stream, lambda: ctx.sha256_fixed_device(d.ptr, 4096, 4096, n, out.ptr, sp))
    res["fixed_4k"] = {"messages": n, "ms": round(ms, 3), "Gblocks_per_s": round(n * 65 / ms / 1e6, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
