"""Where the segment walk's time goes, per segment: a diagnostic build
(EXTRA=-DLSMCK_SEG_CLOCK tools/build_ab.sh D WT, copied over liblsmck.so)
records three wall_clock64 marks per segment (start, after the guess, after
the walk); this replays the framed config-3 log once with the records in HBM
and prints the guess / walk split per lane and per wave (a wave's time is
its slowest lane's).
  python3 tools/seg_clock.py [records]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lsm_storage_engine_amd.device import Context, gen_zipf_lengths, WAL_REC_DTYPE  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    lanes = int(os.environ.get("SEG_CLOCK_LANES", "1"))  # lanes per segment of the build (LSMCK_SEG_GUESS_LANES)
    seg_bytes = int(os.environ.get("SEG_CLOCK_SEG_BYTES", "0"))  # wal_seg_bytes (0: automatic)
    ln = gen_zipf_lengths(0x5EED0003, n)
    off = np.full(n, 13, dtype=np.uint64)
    off[1:] += ln[:-1].astype(np.uint64)
    off = np.cumsum(off, dtype=np.uint64)
    total = int(off[-1]) + int(ln[-1])
    ctx = Context(0)
    d = ctx.alloc(total + 64)
    d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * n)
    ctx.gen_stream(d.ptr, 0x5EED0003, 0, total)
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
    ctx.wal_frame_insert_device(d.ptr, d_o.ptr, d_l.ptr, out.ptr, n, 16)
    ctx.sync()
    rb = ctx.alloc(n * WAL_REC_DTYPE.itemsize)
    ctx.set_option("wal_seg_bytes", seg_bytes)
    for _ in range(3):
        m, st, bad = ctx.wal_replay_verify_to_device(total, rb.ptr, n, device_ptr=d.ptr)
        assert st == 0 and m == n
    K = ctx.get_stat("wal_segments")
    lib = ctx.lib
    buf = np.zeros(3 * 131072, dtype=np.uint64)
    rc = lib.lsmck_diag_seg_clock(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.size))
    assert rc == 0, rc
    K = min(K, 131072)
    t = buf[:3 * K].reshape(K, 3).astype(np.int64)
    t0 = t[:, 0].min()
    guess = (t[:, 1] - t[:, 0]) / 100.0  # us
    walk = (t[:, 2] - t[:, 1]) / 100.0
    end = (t[:, 2] - t0) / 100.0
    per = 64 // lanes  # segments per wave
    W = K // per
    wg = guess[:W * per].reshape(W, per)
    ww = walk[:W * per].reshape(W, per)
    res = {"segments": int(K), "lanes_per_segment": lanes, "seg_bytes": seg_bytes, "kernel_span_us": float(end.max()),
           "lane_guess_us": {"mean": float(guess.mean()), "p50": float(np.median(guess)), "p99": float(np.percentile(guess, 99)), "max": float(guess.max())},
           "lane_walk_us": {"mean": float(walk.mean()), "p50": float(np.median(walk)), "p99": float(np.percentile(walk, 99)), "max": float(walk.max())},
           "wave_max_guess_us": {"mean": float(wg.max(1).mean()), "p50": float(np.median(wg.max(1)))},
           "wave_max_walk_us": {"mean": float(ww.max(1).mean()), "p50": float(np.median(ww.max(1)))},
           "wave_max_guess_plus_walk_us": {"mean": float((wg + ww).max(1).mean())},
           "start_spread_us": float((t[:, 0].max() - t0) / 100.0)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
