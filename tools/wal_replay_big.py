#!/usr/bin/env python3
"""Full-size WAL replay verify on the GPU (SURVEY 8f row 1 at config 3's scale).

Config 3's 2^26 Zipf payloads framed as wal.rs Insert records (a 13-byte
header before each, CRCs written on the device: lsmck_wal_frame_insert_device),
a 97.8 GiB log resident in HBM, replayed by lsmck_wal_replay_verify: the
segment walk of the headers on the GPU (lsmck_segwalk.h), the payload CRC
pass on the stream kernel, the compare, and the 2^26 record descriptors
copied back to the host (into a page-locked array: LSMCK_RECS_PINNED).
--device-recs 1 adds the same replays with the records left in HBM
(LSMCK_RECS_DEVICE), --seg-sweep a segment-size A/B of those.  Every step
checks the record count and the CRC summary against the oracle's
(tests/golden/summaries.json config3w), then prints one JSON line.
--compact 1: the records in the 16-byte form (lsmck_wal_replay_verify16):
they carry no stored CRC, so every step checks every record against the
framing instead (payload offset, Insert, klen = min(len, 16), vlen = the
rest), the replay's status covering the CRCs; --dma-engines sets the SDMA
engines of the read-back (0: hipMemcpyAsync).

--shape mib / logs: the walk's hard logs at full size instead (DESIGN.md
7a): every value ~1 MiB (each segment's first record longer than kHop), or
a log of logs (every value a framed WAL image of 113 B-8 KiB records: the
guesses inside values follow plausible chains that are not the log's).
Their records are checked against their framing (every one, both layouts).

  python3 tools/wal_replay_big.py [--steps 3] [--records 67108864] [--device-recs 1]
(LSMCK_WAL_TRACE=1 prints the replay's phases to stderr.)"""
import argparse
import json
import os
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (before the library: the torch wheel's HIP runtime)
from lsm_storage_engine_amd.device import Context, gen_zipf_lengths  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--records", type=int, default=1 << 26)
    ap.add_argument("--seg-walk", type=int, default=1, help="0: the candidate-doubling walk (A/B)")
    ap.add_argument("--seg-pack", type=int, default=1, help="0: the CRC pass over payloads alone (A/B)")
    ap.add_argument("--seg-stage", type=int, default=1,
                    help="0: no record staging in the walk (the emit walks the headers again; A/B)")
    ap.add_argument("--pinned-recs", type=int, default=1,
                    help="1: the records DMA'd into a page-locked array (LSMCK_RECS_PINNED); 0: staged + copied")
    ap.add_argument("--device-recs", type=int, default=0,
                    help="1: then the same replays with the records left in device memory (LSMCK_RECS_DEVICE)")
    ap.add_argument("--seg-sweep", default="",
                    help="comma list of wal_seg_bytes: the records-on-device replay per segment size (A/B)")
    ap.add_argument("--raw-reps", type=int, default=0,
                    help="A/B: time the plain batch CRC (lsmck_crc32_device) over the framed log's packed spans "
                         "and over its payloads alone, this many times each, before the replays")
    ap.add_argument("--compact", type=int, default=0, help="1: 16-byte records (lsmck_wal_replay_verify16)")
    ap.add_argument("--dma-engines", type=int, default=-1, help="wal_dma_engines (-1: the default)")
    ap.add_argument("--shape", default="zipf", choices=["zipf", "mib", "logs"],
                    help="zipf: config 3's records framed; mib: ~1 MiB values; logs: values that are WAL images")
    ap.add_argument("--log-gib", type=float, default=97.8, help="mib / logs: the log's size")
    ap.add_argument("--opt", action="append", default=[], help="key=value: a context option for every replay")
    ap.add_argument("--variants", default="",
                    help="A/B after the replays: 'name:key=val,key=val;name2:...' -- each variant's options set in "
                         "turn, --ab-rounds interleaved rounds, records to the pinned host array and in HBM")
    ap.add_argument("--ab-rounds", type=int, default=3)
    a = ap.parse_args()
    n = a.records
    inner = None
    if a.shape == "zipf":
        ln = gen_zipf_lengths(0x5EED0003, n)
    else:
        rng = np.random.default_rng(0x5EED0005)
        target = int(a.log_gib * GIB)
        if a.shape == "mib":
            n = target // ((1 << 20) + 2048 + 13)
            ln = ((1 << 20) + rng.integers(0, 4096, n)).astype(np.uint32)
        else:
            n = target // ((1 << 20) + 13)
            ln = rng.integers(256 << 10, 1792 << 10, n).astype(np.uint32)
    off = np.full(n, 13, dtype=np.uint64)
    off[1:] += ln[:-1].astype(np.uint64)
    off = np.cumsum(off, dtype=np.uint64)
    total = int(off[-1]) + int(ln[-1])
    if a.shape == "logs":  # each value: inner records (13-byte header + 100..8000 bytes) filling it exactly
        io, il = [], []
        for o, v in zip(off.tolist(), ln.tolist()):
            sz = rng.integers(113, 8013, v // 3000 + 16)  # (enough draws to pass v)
            cs = np.cumsum(sz)
            k = int(np.searchsorted(cs, v))  # records [0, k] reach v: the last one is cut to fit
            sz = sz[:k + 1].copy()
            sz[k] = v - (int(cs[k - 1]) if k else 0)
            if sz[k] < 13:  # (too short for a header: folded into the one before)
                sz[k - 1] += sz[k]
                sz = sz[:k]
            st = o + np.concatenate(([0], np.cumsum(sz)[:-1]))
            io.append(st + 13)
            il.append(sz - 13)
        inner = (np.concatenate(io).astype(np.uint64), np.concatenate(il).astype(np.uint32))
        print(f"log of logs: {n} values, {len(inner[0])} inner records", file=sys.stderr, flush=True)
    golden = None
    if a.shape == "zipf" and n == 1 << 26:
        with open(os.path.join(ROOT, "tests", "golden", "summaries.json")) as f:
            golden = json.load(f)["config3w"]
        assert total == golden["image_bytes"]
    ctx = Context(0)
    ctx.set_option("wal_seg_walk", a.seg_walk)
    ctx.set_option("wal_seg_pack", a.seg_pack)
    ctx.set_option("wal_seg_stage", a.seg_stage)
    if a.dma_engines >= 0:
        ctx.set_option("wal_dma_engines", a.dma_engines)
    for kv in a.opt:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    kl = np.minimum(ln, 16).astype(np.uint32)  # the framing's key / value split (lsmck_wal_frame_insert_device)

    def check_compact(recs):  # every record against the framing
        assert (recs["payload_type"] == off).all() and (recs["klen"] == kl).all() and (recs["vlen"] == ln - kl).all()

    def check_wide(recs):
        assert (recs["payload_off"] == off).all() and (recs["rec_off"] == off - np.uint64(13)).all()
        assert (recs["klen"] == kl).all() and (recs["vlen"] == ln - kl).all() and (recs["type"] == 1).all()
    d = ctx.alloc(total + 64)
    d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * n)
    ctx.gen_stream(d.ptr, 0x5EED0003, 0, total)
    if inner is not None:  # the inner logs' headers first: the values' CRCs cover them
        ni = len(inner[0])
        i_o, i_l, i_c = ctx.alloc(8 * ni), ctx.alloc(4 * ni), ctx.alloc(4 * ni)
        i_o.upload(inner[0])
        i_l.upload(inner[1])
        ctx.crc32_device(d.ptr, i_o.ptr, i_l.ptr, ni, i_c.ptr)
        ctx.wal_frame_insert_device(d.ptr, i_o.ptr, i_l.ptr, i_c.ptr, ni, 16)
        ctx.sync()
        for b in (i_o, i_l, i_c):
            b.free()
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
    ctx.wal_frame_insert_device(d.ptr, d_o.ptr, d_l.ptr, out.ptr, n, 16)
    ctx.sync()
    raw = {}
    lp = ln.astype(np.uint32).copy()
    lp[:-1] += 13  # [payload | next header)

    def raw_batch(name, lens, key):
        d_l.upload(lens)
        ts = []
        for _ in range(a.raw_reps + 1):
            ctx.sync()
            t = time.perf_counter()
            ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
            ctx.sync()
            ts.append(time.perf_counter() - t)
        raw[key] = round(float(np.median(ts[1:])) * 1e3, 2)
        print(f"raw batch CRC over {name}: {raw[key]} ms", file=sys.stderr, flush=True)
    if a.raw_reps:
        raw_batch("packed spans", lp, "packed_spans")
        raw_batch("payloads", ln, "payloads")
    times = []
    for s in range(a.steps + 1):  # the first replay is a warm-up
        ctx.sync()
        t = time.perf_counter()
        recs, st, bad = ctx.wal_replay_verify(total, device_ptr=d.ptr, cap=n, pinned_recs=bool(a.pinned_recs),
                                              compact=bool(a.compact))
        dt = time.perf_counter() - t
        assert st == 0 and len(recs) == n, (st, len(recs), bad)
        if a.compact:
            check_compact(recs)
            summary = "every record = the framing"
        elif a.shape != "zipf":
            check_wide(recs)
            summary = "every record = the framing"
        else:
            summary = "%08x" % zlib.crc32(np.ascontiguousarray(recs.crc).astype("<u4").tobytes())
            if golden:
                assert summary == golden["summary_crc32"], summary
        if s:
            times.append(dt)
        print(f"replay {s}: {dt * 1e3:.1f} ms (walk path {ctx.get_stat('wal_walk_path')}, "
              f"{ctx.get_stat('wal_segments')} segments, {ctx.get_stat('wal_seg_prepairs')} parallel rounds, "
              f"{ctx.get_stat('wal_seg_repairs')} repairs)",
              file=sys.stderr, flush=True)
        del recs  # the wrapper reuses its records array once no result refers to it
    # the engines of the host-record replays' read-back, read before the
    # records-on-device replays below (which read nothing back: the stat is 0)
    host_dma = ctx.get_stat("wal_recs_dma")
    host_stats = {k: ctx.get_stat(k) for k in ("wal_walk_path", "wal_seg_repairs", "wal_seg_prepairs", "wal_segments",
                                               "wal_pipe_parts")}
    dev = None
    if a.device_recs:  # the records stay in HBM: the walk, the CRC pass and the compare, no host link
        from lsm_storage_engine_amd.device import WAL_REC16_DTYPE, WAL_REC_DTYPE
        RD = WAL_REC16_DTYPE if a.compact else WAL_REC_DTYPE
        rb = ctx.alloc(n * RD.itemsize)
        dts = []
        for s in range(a.steps + 1):
            ctx.sync()
            t = time.perf_counter()
            m, st, bad = ctx.wal_replay_verify_to_device(total, rb.ptr, n, device_ptr=d.ptr, compact=bool(a.compact))
            dt = time.perf_counter() - t
            assert st == 0 and m == n, (st, m, bad)
            if s:
                dts.append(dt)
            print(f"replay (records on the device) {s}: {dt * 1e3:.1f} ms", file=sys.stderr, flush=True)
        sweep = {}
        for sb in [int(x) for x in a.seg_sweep.split(",") if x]:
            ctx.set_option("wal_seg_bytes", sb)
            ts = []
            for s in range(a.steps + 1):
                ctx.sync()
                t = time.perf_counter()
                m, st, bad = ctx.wal_replay_verify_to_device(total, rb.ptr, n, device_ptr=d.ptr, compact=bool(a.compact))
                dt = time.perf_counter() - t
                assert st == 0 and m == n, (st, m, bad)
                if s:
                    ts.append(dt)
            sweep[sb] = {"ms_median": round(float(np.median(ts)) * 1e3, 2), "segments": ctx.get_stat("wal_segments"),
                         "repairs": ctx.get_stat("wal_seg_repairs"), "path": ctx.get_stat("wal_walk_path")}
            print(f"wal_seg_bytes {sb}: {sweep[sb]}", file=sys.stderr, flush=True)
        ctx.set_option("wal_seg_bytes", 0)
        if a.raw_reps:  # the same batch again after the replays (order effects)
            raw_batch("packed spans, after the replays", lp, "packed_spans_after")
        got = rb.download(np.uint8, n * RD.itemsize).view(RD)
        if a.compact:
            check_compact(got)
            dsum = "every record = the framing"
        elif a.shape != "zipf":
            check_wide(got)
            dsum = "every record = the framing"
        else:
            dsum = "%08x" % zlib.crc32(np.ascontiguousarray(got["crc"]).astype("<u4").tobytes())
        rb.free()
        dmed = float(np.median(dts))
        dev = {"ms_median": round(dmed * 1e3, 2), "ms_best": round(min(dts) * 1e3, 2),
               "value": round(total / GIB / dmed, 1), "summary_crc32": dsum,
               # (as the host line's: compact and non-Zipf records are each checked against the framing)
               "summary_matches_oracle": bool(a.compact) or a.shape != "zipf" or (bool(golden) and dsum == golden["summary_crc32"]),
               "seg_sweep": sweep}
    ab = {}
    if a.variants:  # interleaved A/B of option sets: records to the pinned host array, then in HBM
        from lsm_storage_engine_amd.device import WAL_REC16_DTYPE, WAL_REC_DTYPE
        RD = WAL_REC16_DTYPE if a.compact else WAL_REC_DTYPE
        rb = ctx.alloc(n * RD.itemsize)
        vs = []
        for item in a.variants.split(";"):
            name, _, kvs = item.partition(":")
            vs.append((name, [(k, int(v)) for k, v in (kv.split("=") for kv in kvs.split(",") if kv)]))
        # (every variant names the options it sets; a key one variant sets and another does not keeps the last value)
        res = {name: {"host": [], "dev": [], "parts": None} for name, _ in vs}
        for r in range(a.ab_rounds + 1):  # (round 0: warm-up)
            for name, o in vs:
                for k, v in o:
                    ctx.set_option(k, v)
                ctx.sync()
                t = time.perf_counter()
                recs, st, bad = ctx.wal_replay_verify(total, device_ptr=d.ptr, cap=n, pinned_recs=bool(a.pinned_recs),
                                                      compact=bool(a.compact))
                th = time.perf_counter() - t
                assert st == 0 and len(recs) == n, (name, st, len(recs), bad)
                if a.compact:
                    check_compact(recs)
                elif a.shape != "zipf":
                    check_wide(recs)
                del recs
                ctx.sync()
                t = time.perf_counter()
                m, st, bad = ctx.wal_replay_verify_to_device(total, rb.ptr, n, device_ptr=d.ptr, compact=bool(a.compact))
                td = time.perf_counter() - t
                assert st == 0 and m == n, (name, st, m, bad)
                if r:
                    res[name]["host"].append(th)
                    res[name]["dev"].append(td)
                res[name]["parts"] = ctx.get_stat("wal_pipe_parts")
                print(f"ab round {r} {name}: host {th * 1e3:.2f} ms, HBM {td * 1e3:.2f} ms, "
                      f"{res[name]['parts']} parts", file=sys.stderr, flush=True)
            got = rb.download(np.uint8, n * RD.itemsize).view(RD)
            if a.compact:
                check_compact(got)
            elif a.shape != "zipf":
                check_wide(got)
        rb.free()
        for name, v in res.items():
            ab[name] = {"host_ms_median": round(float(np.median(v["host"])) * 1e3, 2),
                        "dev_ms_median": round(float(np.median(v["dev"])) * 1e3, 2),
                        "host_ms": [round(x * 1e3, 2) for x in v["host"]],
                        "dev_ms": [round(x * 1e3, 2) for x in v["dev"]], "pipe_parts": v["parts"]}
    for b in (d_o, d_l, out):
        b.free()
    d.free()
    best, med = min(times), float(np.median(times))
    print(json.dumps({
        "metric": "WAL replay verify of a device-resident log (header walk + payload CRC check + records to host)",
        "value": round(total / GIB / med, 1), "unit": "GiB/s of log",
        "log_bytes": total, "records": n, "ms_median": round(med * 1e3, 2), "ms_best": round(best * 1e3, 2),
        "steps": a.steps, "summary_crc32": summary,
        "summary_matches_oracle": bool(golden) or a.shape != "zipf" or bool(a.compact), "shape": a.shape,
        "records_out_bytes": (16 if a.compact else 32) * n, "pinned_recs": bool(a.pinned_recs),
        "compact": bool(a.compact), "recs_dma_engines": host_dma,
        "walk_path": {1: "segment walk", 2: "candidate doubling", 3: "host walk"}.get(host_stats["wal_walk_path"]),
        "seg_repairs": host_stats["wal_seg_repairs"], "seg_prepairs": host_stats["wal_seg_prepairs"],
        "segments": host_stats["wal_segments"], "pipe_parts": host_stats["wal_pipe_parts"], "options": a.opt,
        "variants_ab": ab,
        "records_on_device": dev, "raw_batch_crc_ms": raw,
        "workload": {"zipf": "config 3's 2^26 Zipf payloads (64 B-64 KiB) framed as wal.rs Insert records "
                             "(13-byte headers), headers and CRCs written on the device",
                     "mib": f"{n} Insert records of 1 MiB + 0..4095 B values, random bytes",
                     "logs": f"{n} Insert records whose values (256 KiB-1.75 MiB) are WAL images of "
                             f"{0 if inner is None else len(inner[0])} framed records of 100-8000 B"}[a.shape]}))


if __name__ == "__main__":
    main()
