"""Where the WAL replay verify's time goes (config 5's WAL leg).

Builds a WAL image like tree.synthesize_tree's (500k records, keys 1-39 B,
values 0-999 B, 10% removes), then times, best of 5 each:
  replay    lsmck_wal_replay_verify: by default a host image is uploaded and
            walked on the GPU; the host walk (wal_upload_min 0) is timed too, and
            per wal_prefetch distance (A/B of the walk's prefetch) and per
            wal_chunk_bytes (CRC batches overlapped with the walk; 0 = one
            batch after it)
  verify    lsmck_crc32_verify_batch on the same descriptors, pageable host image
  pinned    the same from a pinned copy of the image
  device    the same on a device-resident copy; replay of a device-resident
            image with the GPU header walk (default) and with the copy-back
            host walk (wal_gpu_walk 0)
Prints one JSON line.
"""
import json
import os
import struct
import sys
import time
import zlib

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


def build_image(n, with_descriptors=False):
    """tree.synthesize_tree's WAL shape: keys 1-39 B, values 0-999 B, 10% removes."""
    rng = np.random.default_rng(5)
    pool = rng.bytes(1 << 20)
    kl = rng.integers(1, 40, size=n)
    vl = rng.integers(0, 1000, size=n)
    rm = rng.random(n) < 0.1
    wal = bytearray()
    off, ln, exp = [], [], []
    for i in range(n):
        o = (i * 7919) % ((1 << 20) - 1100)
        key = pool[o:o + int(kl[i])]
        d = key if rm[i] else key + pool[o + 40:o + 40 + int(vl[i])]
        hdr = struct.pack("<BII", 2, zlib.crc32(d), len(key)) if rm[i] else \
            struct.pack("<BIII", 1, zlib.crc32(d), len(key), int(vl[i]))
        wal += hdr
        off.append(len(wal))
        ln.append(len(d))
        exp.append(zlib.crc32(d))
        wal += d
    img = np.frombuffer(bytes(wal), dtype=np.uint8)
    if not with_descriptors:
        return img
    return img, np.array(off, dtype=np.uint64), np.array(ln, dtype=np.uint32), np.array(exp, dtype=np.uint32)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000
    img, off, ln, exp = build_image(n, True)
    ctx = Context(0)
    res = {"wal_bytes": len(img), "records": n}
    recs, st, _ = ctx.wal_replay_verify(img)
    assert st == 0 and len(recs) == n
    res["replay_total_s"] = best(lambda: ctx.wal_replay_verify(img))  # default: uploaded, GPU header walk
    # the same through the C ABI into one records array reused across calls
    # (the wrapper allocates a worst-case n/9-record array per call)
    import ctypes as C
    from lsm_storage_engine_amd import _lib
    from lsm_storage_engine_amd.device import WAL_REC_DTYPE
    rbuf = np.empty(len(img) // 9 + 1, dtype=WAL_REC_DTYPE)
    out = (C.c_size_t(), C.c_uint64(), C.c_uint32(), C.c_uint32())

    def reuse():
        rc = ctx.lib.lsmck_wal_replay_verify(ctx.handle, img.ctypes.data, len(img), _lib.HOST, rbuf.ctypes.data,
                                             len(rbuf), *[C.byref(x) for x in out])
        assert rc == 0 and out[0].value == n
    res["replay_reuse_recs_s"] = best(reuse)
    ctx.set_option("wal_split", 0)  # A/B: the whole image uploaded before the walk
    res["replay_nosplit_s"] = best(lambda: ctx.wal_replay_verify(img))
    ctx.set_option("wal_split", 1)
    for sb in (4, 8, 32, 64):  # A/B: upload chunk size (pipeline fill / drain against per-chunk cost)
        ctx.set_option("wal_stage_bytes", sb << 20)
        res[f"replay_stage_{sb}MiB_s"] = best(lambda: ctx.wal_replay_verify(img))
    ctx.set_option("wal_stage_bytes", 16 << 20)
    ctx.set_option("wal_register", 1)  # A/B: the caller's pages pinned in place, DMA without the staging copy
    res["replay_registered_s"] = best(lambda: ctx.wal_replay_verify(img))
    ctx.set_option("wal_register", 0)
    ctx.set_option("wal_upload_min", 0)  # the host walk for the A/Bs below
    res["replay_hostwalk_s"] = best(lambda: ctx.wal_replay_verify(img))
    for pf in (0, 1024, 4096, 16384, 65536):
        ctx.set_option("wal_prefetch", pf)
        res[f"replay_prefetch_{pf}_s"] = best(lambda: ctx.wal_replay_verify(img))
    ctx.set_option("wal_prefetch", 4096)
    for ch in (0, 8 << 20, 32 << 20, 64 << 20):
        ctx.set_option("wal_chunk_bytes", ch)
        res[f"replay_chunk_{ch >> 20}MiB_s"] = best(lambda: ctx.wal_replay_verify(img))
    ctx.set_option("wal_chunk_bytes", 32 << 20)
    for th in (1, 4, 8, 16):
        ctx.set_option("stage_threads", th)
        res[f"verify_pageable_stage{th}_s"] = best(lambda: ctx.crc32_verify(img, off, ln, exp))
        res[f"replay_stage{th}_s"] = best(lambda: ctx.wal_replay_verify(img))
    ctx.set_option("stage_threads", 8)
    res["verify_pageable_s"] = best(lambda: ctx.crc32_verify(img, off, ln, exp))
    pin = ctx.alloc_pinned(len(img))
    pin.array[:] = img
    res["replay_pinned_image_hostwalk_s"] = best(lambda: ctx.wal_replay_verify(pin.array))
    ctx.set_option("wal_upload_min", 1 << 20)
    res["replay_pageable_upload_gpuwalk_s"] = best(lambda: ctx.wal_replay_verify(img))
    d = ctx.alloc(len(img))
    d.upload(img)
    ctx.sync()
    res["replay_device_image_s"] = best(lambda: ctx.wal_replay_verify(len(img), device_ptr=d.ptr))
    # the records DMA'd into a page-locked array (LSMCK_RECS_PINNED), cap = the record count
    res["replay_device_image_pinned_recs_s"] = best(
        lambda: ctx.wal_replay_verify(len(img), device_ptr=d.ptr, cap=n, pinned_recs=True))
    res["device_walk_path"] = ctx.get_stat("wal_walk_path")
    res["device_segments"] = ctx.get_stat("wal_segments")
    res["device_seg_repairs"] = ctx.get_stat("wal_seg_repairs")
    ctx.set_option("wal_seg_walk", 0)  # A/B: candidate doubling
    res["replay_device_image_doubling_s"] = best(lambda: ctx.wal_replay_verify(len(img), device_ptr=d.ptr))
    ctx.set_option("wal_seg_walk", 1)
    ctx.set_option("wal_gpu_walk", 0)  # A/B: copy the device image back, host walk
    res["replay_device_image_hostwalk_s"] = best(lambda: ctx.wal_replay_verify(len(img), device_ptr=d.ptr))
    ctx.set_option("wal_gpu_walk", 1)
    # a host image uploaded whole from pinned memory, then the GPU header walk
    res["replay_pinned_upload_gpuwalk_s"] = best(
        lambda: (d.upload(pin.array), ctx.wal_replay_verify(len(img), device_ptr=d.ptr)))
    for k in list(res):
        if k.endswith("_s") and isinstance(res[k], float):
            res[k[:-2] + "_GiBps"] = round(len(img) / 2**30 / res[k], 2)
            res[k] = round(res[k], 4)
    print(json.dumps(res))
    d.free()
    pin.free()
    ctx.close()


if __name__ == "__main__":
    main()
