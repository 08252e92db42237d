"""The default WAL replay (host image: upload + GPU header walk + CRC pass)
and the device-image replay, ten times each, for a kernel trace:
  rocprofv3 --kernel-trace --stats -d gpurun_out/kt_wal -o kt -- python3 tools/wal_kt.py
Same image as tools/wal_diag.py (500k records, 0.24 GB)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lsm_storage_engine_amd.device import Context  # noqa: E402
import wal_diag  # noqa: E402


def main():
    img = wal_diag.build_image(500_000)
    ctx = Context(0)
    out = {}
    for name, fn in (("host_image", lambda: ctx.wal_replay_verify(img)),):
        fn()
        ts = []
        for _ in range(10):
            t = time.perf_counter()
            recs, st, _ = fn()
            ts.append(time.perf_counter() - t)
            assert st == 0 and len(recs) == 500_000
        out[name + "_ms_best"] = round(min(ts) * 1e3, 3)
    d = ctx.alloc(len(img))
    d.upload(img)
    ctx.sync()
    ts = []
    for _ in range(10):
        t = time.perf_counter()
        recs, st, _ = ctx.wal_replay_verify(len(img), device_ptr=d.ptr)
        ts.append(time.perf_counter() - t)
    out["device_image_ms_best"] = round(min(ts) * 1e3, 3)
    ts = []  # the records DMA'd into a page-locked array (LSMCK_RECS_PINNED)
    for _ in range(11):
        t = time.perf_counter()
        recs, st, _ = ctx.wal_replay_verify(len(img), device_ptr=d.ptr, cap=500_000, pinned_recs=True)
        ts.append(time.perf_counter() - t)
        assert st == 0 and len(recs) == 500_000
        del recs
    out["device_image_pinned_recs_ms_best"] = round(min(ts[1:]) * 1e3, 3)
    out["device_image_pinned_recs_ms_median"] = round(float(np.median(ts[1:])) * 1e3, 3)
    from lsm_storage_engine_amd.device import WAL_REC_DTYPE
    rb = ctx.alloc(500_000 * WAL_REC_DTYPE.itemsize)
    ts = []  # the records left in device memory (LSMCK_RECS_DEVICE; builds before it: WAL_KT_DEVRECS=0)
    for _ in range(11 if os.environ.get("WAL_KT_DEVRECS", "1") != "0" else 0):
        t = time.perf_counter()
        m, st, _ = ctx.wal_replay_verify_to_device(len(img), rb.ptr, 500_000, device_ptr=d.ptr)
        ts.append(time.perf_counter() - t)
        assert st == 0 and m == 500_000
    for sb in [int(x) for x in os.environ.get("WAL_KT_SEGS", "").split(",") if x]:  # A/B: segment sizes
        ctx.set_option("wal_seg_bytes", sb)
        tt = []
        for _ in range(11):
            t = time.perf_counter()
            m, st, _ = ctx.wal_replay_verify_to_device(len(img), rb.ptr, 500_000, device_ptr=d.ptr)
            tt.append(time.perf_counter() - t)
            assert st == 0 and m == 500_000
        out[f"device_recs_seg{sb}_ms_median"] = round(float(np.median(tt[1:])) * 1e3, 3)
        out[f"device_recs_seg{sb}_repairs"] = ctx.get_stat("wal_seg_repairs")
    ctx.set_option("wal_seg_bytes", 0)
    rb.free()
    if ts:
        out["device_image_device_recs_ms_best"] = round(min(ts[1:]) * 1e3, 3)
        out["device_image_device_recs_ms_median"] = round(float(np.median(ts[1:])) * 1e3, 3)
    out["walk"] = {"path": ctx.get_stat("wal_walk_path"), "segments": ctx.get_stat("wal_segments"),
                   "repairs": ctx.get_stat("wal_seg_repairs")}
    print(out)
    d.free()
    ctx.close()


if __name__ == "__main__":
    main()
