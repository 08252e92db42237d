#!/usr/bin/env python3
"""BASELINE config 5, end to end: the checksum work of Db::load over an LSM tree
on disk -- every SSTable's data + index file SHA-256-verified against its
checksum file, and the WAL replayed with every record's CRC-32 checked
(lsm_storage_engine_amd/tree.py; src/tokio/db.rs:37-73).

  python3 tools/e2e_tree.py [--gib 16] [--dir /tmp/lsm_e2e] [--reps 3] [--keep]

Writes a synthetic tree in the reference's on-disk layout (if --dir does not
already hold one), then times load_verify() --reps times with the page cache
warm (the tree was just written; dropping caches needs root, which the GPU box
does not give).  Prints one JSON line.  The rate includes reading the files
(16 reader threads, pread), the PCIe copies and the GPU batches; it is not a
device-resident number.  A CPU baseline (the oracle's FIPS SHA-256, one
thread, on the first tables) is timed beside it.
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np
import torch  # noqa: F401  (first: liblsmck binds to torch's HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lsm_storage_engine_amd.device import Context  # noqa: E402
from lsm_storage_engine_amd import tree  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=16.0, help="SSTable data bytes of the tree (GiB)")
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "lsm_e2e"))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--wal-records", type=int, default=500_000)
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--cpu-sample-gib", type=float, default=1.0)
    ap.add_argument("--list-threads", default="", help="comma list of tree_list_threads values to A/B (listing time)")
    ap.add_argument("--ab", default="", help="comma list of active:slice_bytes[:open_files] settings to A/B after the main reps")
    ap.add_argument("--stages", default="",
                    help="comma list of tree_stages values to A/B (interleaved, 3 rounds each): the verify's seconds")
    ap.add_argument("--overlap", default="",
                    help="comma list of tree_overlap values to A/B (interleaved, 3 rounds each): list + verify seconds")
    ap.add_argument("--tick", default="",
                    help="comma list of tree_json_threads[:tree_active_files] values: the compaction tick's batch (levels 0..3 through "
                         "lsmck_checksums_verify_many), interleaved, 3 rounds each")
    ap.add_argument("--readers", default="",
                    help="comma list of tree_readers values: the tree verify and the compaction tick's batch per "
                         "value, interleaved, 3 rounds")
    ap.add_argument("--multi", type=int, default=0,
                    help="also time lsmck_tree_verify_multi with this many contexts on device 0 against "
                         "lsmck_tree_verify on one (the multi-GPU split's own cost, measurable on one GPU)")
    a = ap.parse_args()

    marker = os.path.join(a.dir, "e2e_tree.json")
    if os.path.exists(marker):
        with open(marker) as f:
            synth = json.load(f)
    else:
        shutil.rmtree(a.dir, ignore_errors=True)
        os.makedirs(a.dir)
        synth = tree.synthesize_tree(a.dir, int(a.gib * GIB), wal_records=a.wal_records,
                                     progress=lambda m: print(m, file=sys.stderr, flush=True))
        with open(marker, "w") as f:
            json.dump(synth, f)
    print(f"tree: {synth}", file=sys.stderr, flush=True)

    ctx = Context(0)
    reports = []
    for r in range(a.reps):
        mem, rep = tree.load_verify(ctx, a.dir)
        reports.append(rep)
        print(f"rep {r}: {rep}", file=sys.stderr, flush=True)
    best = min(reports, key=lambda x: x["total_s"])
    ab = {}
    for v in filter(None, a.ab.split(",")):
        act, sl, op = ([int(x) for x in v.split(":")] + [-1])[:3]
        ctx.set_option("tree_active_files", act)
        ctx.set_option("tree_slice_bytes", sl)
        ctx.set_option("tree_open_files", op)
        t = min(tree.load_verify(ctx, a.dir)[1]["tables_s"] for _ in range(2))
        ab[v] = round(best["table_bytes"] / GIB / t, 2)
        print(f"ab {v}: {ab[v]} GiB/s", file=sys.stderr, flush=True)
    ctx.set_option("tree_active_files", 0)
    ctx.set_option("tree_slice_bytes", 0)
    ctx.set_option("tree_open_files", -1)
    lt = {}
    for v in filter(None, a.list_threads.split(",")):
        ctx.set_option("tree_list_threads", int(v))
        lt[v] = round(min(tree.load_verify(ctx, a.dir)[1]["list_s"] for _ in range(2)), 3)
        print(f"list threads {v}: {lt[v]} s", file=sys.stderr, flush=True)
    ctx.set_option("tree_list_threads", 0)
    stages = {}
    for _ in range(3 if a.stages else 0):
        for v in filter(None, a.stages.split(",")):
            ctx.set_option("tree_stages", int(v))
            r = tree.load_verify(ctx, a.dir)[1]
            stages.setdefault(v, []).append({"tables_s": round(r["tables_s"], 3), **{
                k: round(x, 3) for k, x in r["tables_split"].items() if isinstance(x, float)}})
            print(f"stages {v}: {stages[v][-1]}", file=sys.stderr, flush=True)
    ctx.set_option("tree_stages", 3)
    overlap = {}
    for _ in range(3 if a.overlap else 0):
        for v in filter(None, a.overlap.split(",")):
            ctx.set_option("tree_overlap", int(v))
            r = tree.load_verify(ctx, a.dir)[1]
            overlap.setdefault(v, []).append({"list_s": round(r["list_s"], 3), "tables_s": round(r["tables_s"], 3),
                                              "list_plus_tables_s": round(r["list_s"] + r["tables_s"], 3)})
            print(f"overlap {v}: {overlap[v][-1]}", file=sys.stderr, flush=True)
    ctx.set_option("tree_overlap", 2048)
    tick = {}
    if a.tick:
        low = [m for m in tree.list_tables(a.dir) if m.level <= 3]
        triples = [(m.data_path(), m.index_path(), m.checksum_path()) for m in low]
        nbytes = sum(os.path.getsize(x) + os.path.getsize(y) for x, y, _ in triples)
        for _ in range(3):
            for v in filter(None, a.tick.split(",")):
                jt, act = ([int(x) for x in v.split(":")] + [0])[:2]  # json threads[:active files]
                ctx.set_option("tree_json_threads", jt)
                ctx.set_option("tree_active_files", act)
                t = time.perf_counter()
                st = ctx.checksums_verify_many(triples)
                dt = time.perf_counter() - t
                assert not any(st)
                tick.setdefault(v, []).append(round(dt, 3))
                print(f"tick json threads[:active] {v}: {len(triples)} tables, {nbytes / GIB:.2f} GiB, {dt:.3f} s",
                      file=sys.stderr, flush=True)
        ctx.set_option("tree_json_threads", 0)
        ctx.set_option("tree_active_files", 0)
    readers = {}
    if a.readers:
        low = [m for m in tree.list_tables(a.dir) if m.level <= 3]
        triples = [(m.data_path(), m.index_path(), m.checksum_path()) for m in low]
        for _ in range(3):
            for v in filter(None, a.readers.split(",")):
                ctx.set_option("tree_readers", int(v))
                r = tree.load_verify(ctx, a.dir)[1]
                t = time.perf_counter()
                st = ctx.checksums_verify_many(triples)
                dt = time.perf_counter() - t
                assert not any(st)
                e = readers.setdefault(v, {"tables_s": [], "tick_s": [], "read_s": []})
                e["tables_s"].append(round(r["tables_s"], 3))
                e["read_s"].append(round(r["tables_split"]["read_seconds"], 3))
                e["tick_s"].append(round(dt, 3))
                print(f"readers {v}: tree verify {r['tables_s']:.3f} s, tick batch {dt:.3f} s", file=sys.stderr,
                      flush=True)
        ctx.set_option("tree_readers", 16)
    multi = None
    if a.multi > 1:
        from lsm_storage_engine_amd.device import MultiContext
        mc = MultiContext(contexts=[Context(0) for _ in range(a.multi)])
        one, many = [], []
        for _ in range(3):  # interleaved
            t = time.perf_counter()
            r1 = ctx.tree_verify(a.dir)
            one.append(time.perf_counter() - t)
            t = time.perf_counter()
            rm = mc.tree_verify(a.dir)
            many.append(time.perf_counter() - t)
            assert r1["bad_tables"] == rm["bad_tables"] == 0 and r1["tables"] == rm["tables"]
        multi = {"contexts_on_one_gpu": a.multi, "tree_verify_s_one_ctx": [round(x, 3) for x in one],
                 "tree_verify_multi_s": [round(x, 3) for x in many],
                 "ratio_median": round(float(np.median(many)) / float(np.median(one)), 3)}
        print(f"multi: {multi}", file=sys.stderr, flush=True)
        for c in mc.ctxs:
            c.close()
    verified = best["table_bytes"] + best["wal_bytes"]

    # CPU baseline: the oracle's SHA-256 (= sha2 0.10's algorithm; scalar, no
    # SHA-NI), one thread, over the first tables' data + index files
    from oracle import oracle as O
    metas = tree.list_tables(a.dir)
    done, t0 = 0, time.perf_counter()
    for m in metas:
        for p in (m.data_path(), m.index_path()):
            O.file_checksum(p)
            done += os.path.getsize(p)
        if done >= a.cpu_sample_gib * GIB:
            break
    tc = time.perf_counter() - t0

    res = {
        "tree_stages_ab": stages or None,
        "tree_overlap_ab": overlap or None,
        "tick_json_threads_ab": tick or None,
        "metric": "GiB/s end-to-end tree load verify (files in the page cache or tmpfs)",
        "value": round(verified / GIB / best["total_s"], 2),
        "unit": "GiB/s",
        "config": {"workload": "config5: Db::load checksum work over a synthetic LSM tree in the reference layout",
                   "tree_tables": best["tables"], "table_bytes": best["table_bytes"], "wal_bytes": best["wal_bytes"],
                   "wal_records": best["wal_records"], "tree_gib": a.gib, "dir": a.dir,
                   "baseline_config": "BASELINE config 5: a 100 GiB tree"},
        "seconds": {k: round(best[k], 3) for k in ("list_s", "tables_s", "wal_s", "memtable_build_s", "total_s")},
        "tables_GiBps": round(best["table_bytes"] / GIB / best["tables_s"], 2),
        "tables_split_s": {k: round(v, 3) if isinstance(v, float) else v for k, v in best["tables_split"].items()},
        "wal_GiBps": round(best["wal_bytes"] / GIB / best["wal_s"], 2),
        "reps": [round(x["total_s"], 3) for x in reports],
        "cpu_baseline": {"value": round(done / GIB / tc, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                         "sample": f"first {done / GIB:.2f} GiB of data+index files, oracle FIPS SHA-256 "
                                   "(Checksums::calculate_checksum's digest), 1 thread"},
        "synthesis_s": synth["seconds"],
    }
    if ab:
        res["tables_GiBps_by_active_slice"] = ab
    if lt:
        res["list_s_by_threads"] = lt
    if multi:
        res["tree_verify_multi_same_gpu"] = multi
    if readers:
        res["tree_readers_ab"] = readers
    print(json.dumps(res), flush=True)
    ctx.close()
    if not a.keep:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
