#!/usr/bin/env python3
"""BASELINE config 5 through the loopback server: "checksum-verify WAL replay +
full SSTable scan of a 100 GiB LSM tree via the loopback server".

  python3 tools/e2e_server.py [--gib 100] [--dir /dev/shm/lsm_e2e] [--ops 200000] [--conns 8]

1. Writes a synthetic tree in the reference's on-disk layout (tree.synthesize_tree)
   with a WAL of --wal-records records, unless --dir holds one already.
2. Starts lsmck_server on it: its start-up is Db::load -- every table verified
   on the GPU (lsmck_tree_verify) and the WAL replayed with every CRC checked
   on the GPU (lsmck_wal_replay_verify).  The server reports the phases.
3. Drives --ops insert / get / delete commands over --conns loopback
   connections (each insert and delete appends a CRC-32-framed WAL record,
   lsmck_crc32_ieee; memtable flushes write SSTables with checksum files).
4. Kills the server with SIGKILL and restarts it: the second start-up verifies
   the grown tree and replays the WAL written by the traffic; every key's value
   read back must match what the traffic left.

Prints one JSON line.  Files live in the page cache / tmpfs (dropping caches
needs root).  A CPU baseline (the oracle's FIPS SHA-256, one thread, on the
first GiB of table files) is timed beside it.
"""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lsm_storage_engine_amd import tree  # noqa: E402
from lsm_storage_engine_amd.server import Client, Server  # noqa: E402

GIB = float(1 << 30)


def traffic(port, conn, ops, batch=512):
    """One connection's commands: inserts of its own keys, reads, deletes."""
    c = Client(port)
    model = {}
    hist = {}  # every value a key held
    t0 = time.perf_counter()
    i = 0
    while i < ops:
        cmds, want = [], []
        for j in range(i, min(ops, i + batch)):
            k = b"c%02dk%07d" % (conn, j % max(1, ops // 3))
            if j % 10 == 9:
                cmds.append(b"delete " + k)
                want.append(b"ok")
                model[k] = None
            elif j % 10 == 5:
                cmds.append(b"get " + k)
                v = model.get(k)
                want.append(v if v is not None else k + b" not found")
            else:
                v = b"v%d" % j
                cmds.append(b"insert " + k + b" " + v)
                want.append(b"ok")
                model[k] = v
                hist.setdefault(k, set()).add(v)
        got = c.pipeline(cmds)
        if conn == 0 and (i // batch) % 50 == 0:
            print(f"traffic: conn 0 at {i}/{ops}", file=sys.stderr, flush=True)
        if got != want:
            bad = next(x for x in range(len(got)) if got[x] != want[x])
            raise AssertionError(f"conn {conn}: {cmds[bad]!r} -> {got[bad]!r}, want {want[bad]!r}")
        i += batch
    dt = time.perf_counter() - t0
    c.close()
    return model, hist, dt


def replayed_removes(base):
    """Keys whose last record in the log the restart replays (a rotated
    wal.log.flushing first, then wal.log) is a Remove (oracle replay)."""
    from oracle import oracle as O
    img = b""
    for name in ("wal.log.flushing", "wal.log"):
        p = os.path.join(base, "wal", name)
        if os.path.exists(p):
            img += open(p, "rb").read()
    st, recs, _ = O.wal_replay(img)
    last = {}
    for r in recs:
        p = img[r.payload_off:r.payload_off + ((r.klen + r.vlen) & 0xFFFFFFFF)]
        if r.type == 1:
            last[p[:r.klen]] = 1
        else:
            last[p] = 2
    return {k for k, t in last.items() if t == 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=100.0)
    ap.add_argument("--dir", default="/dev/shm/lsm_e2e_server")
    ap.add_argument("--wal-records", type=int, default=500_000)
    ap.add_argument("--ops", type=int, default=200_000, help="commands per connection")
    ap.add_argument("--conns", type=int, default=8)
    ap.add_argument("--memtable-limit", type=int, default=4 << 20,
                    help="bytes (the reference's config/default is 4096)")
    ap.add_argument("--cpu-sample-gib", type=float, default=1.0)
    ap.add_argument("--compact-interval", type=int, default=10000,
                    help="ms between the server's compaction ticks (server.rs:94; each re-verifies levels 0..3)")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--load-ab", default="",
                    help="comma list of --index-threads values: more restarts (Db::load only), interleaved, 3 each")
    a = ap.parse_args()

    marker = os.path.join(a.dir, "e2e_tree.json")
    if os.path.exists(marker):
        synth = json.load(open(marker))
    else:
        shutil.rmtree(a.dir, ignore_errors=True)
        os.makedirs(a.dir)
        synth = tree.synthesize_tree(a.dir, int(a.gib * GIB), wal_records=a.wal_records,
                                     progress=lambda m: print(m, file=sys.stderr, flush=True))
        json.dump(synth, open(marker, "w"))
    print(f"tree: {synth}", file=sys.stderr, flush=True)

    t0 = time.perf_counter()
    srv = Server(a.dir, memtable_limit=a.memtable_limit, compact_interval_ms=a.compact_interval)
    start1 = time.perf_counter() - t0
    load1 = srv.loaded
    print(f"first start: {load1}", file=sys.stderr, flush=True)
    t1 = time.perf_counter()
    with cf.ThreadPoolExecutor(a.conns) as ex:
        outs = list(ex.map(lambda k: traffic(srv.port, k, a.ops), range(a.conns)))
    wall = time.perf_counter() - t1
    # the compaction ticks that ran while the traffic did (the first one at once)
    ticks = srv.drain_events("compact")
    if not ticks and a.compact_interval > 0:
        ticks = [srv.wait_event("compact", timeout=600)]
    failed = srv.drain_events("compact_failed")
    print(f"ticks: {ticks} {failed}", file=sys.stderr, flush=True)
    srv.kill()
    model, hist = {}, {}
    for m, h, _ in outs:
        model.update(m)
        hist.update(h)
    removed = replayed_removes(a.dir)
    t0 = time.perf_counter()
    srv = Server(a.dir, memtable_limit=a.memtable_limit)
    start2 = time.perf_counter() - t0
    load2 = srv.loaded
    print(f"restart: {load2}", file=sys.stderr, flush=True)
    c = srv.client()
    keys = sorted(model)
    got = []
    for i in range(0, len(keys), 4096):
        got += c.pipeline([b"get " + k for k in keys[i:i + 4096]])
    want = [model[k] if model[k] is not None else k + b" not found" for k in keys]
    # The reference's MemTable::from_log drops the entry of a replayed Remove
    # (memtable.rs:40-43) instead of keeping the tombstone vec![0] a live
    # delete inserts (db.rs:131-143): after a crash, a key whose delete was
    # only in the log reads as its value in the newest table holding it (or
    # not found).  lsmck_server keeps that behaviour; such keys are counted
    # apart and must read as "not found" or as a value the key once held.
    mismatches = resurrected = 0
    for k, x, y in zip(keys, got, want):
        if x == y:
            continue
        if k in removed and (x == k + b" not found" or x in hist.get(k, ())):
            resurrected += 1
        else:
            mismatches += 1
    c.close()
    srv.kill()
    load_ab = {}
    for _ in range(3 if a.load_ab else 0):
        for v in filter(None, a.load_ab.split(",")):
            s2 = Server(a.dir, memtable_limit=a.memtable_limit, exit_after_load=True, index_threads=int(v))
            ld = s2.loaded
            s2.kill()
            load_ab.setdefault(v, []).append({k: ld[k] for k in ("load_s", "tree_verify_s", "tree_list_s", "index_load_s")})
            print(f"load index threads {v}: {load_ab[v][-1]}", file=sys.stderr, flush=True)

    # CPU baseline: the oracle's SHA-256, one thread, the first tables' files
    from oracle import oracle as O
    done, tc0 = 0, time.perf_counter()
    for m in tree.list_tables(a.dir):
        for p in (m.data_path(), m.index_path()):
            O.file_checksum(p)
            done += os.path.getsize(p)
        if done >= a.cpu_sample_gib * GIB:
            break
    tc = time.perf_counter() - tc0

    verified1 = load1["table_bytes"] + load1["wal_bytes"]
    res = {
        "metric": "GiB/s end-to-end Db::load checksum verify through the loopback server (tables + WAL)",
        "value": round(verified1 / GIB / load1["load_s"], 2),
        "unit": "GiB/s",
        "config": {"workload": "config5: lsmck_server start-up (Db::load) on a synthetic LSM tree in the reference "
                               "layout, then loopback traffic, SIGKILL and restart",
                   "tree_gib": a.gib, "dir": a.dir, "tables": load1["tables"], "table_bytes": load1["table_bytes"],
                   "wal_bytes": load1["wal_bytes"], "wal_records": load1["wal_records"],
                   "memtable_limit_bytes": a.memtable_limit},
        "first_start": {**load1, "process_start_s": round(start1, 3),
                        "tables_GiBps": round(load1["table_bytes"] / GIB / load1["tree_verify_s"], 2)},
        "traffic": {"connections": a.conns, "commands": a.conns * a.ops, "seconds": round(wall, 3),
                    "commands_per_s": round(a.conns * a.ops / wall, 1),
                    "mix": "per connection: 80% insert, 10% get, 10% delete, pipelined 512 per round trip"},
        "restart": {**load2, "process_start_s": round(start2, 3)},
        "load_index_threads_ab": load_ab or None,
        "compaction_ticks": {"interval_ms": a.compact_interval, "ticks_during_traffic": len(ticks),
                             "what": "Db::compact's re-verify of levels 0..3 (SsTable::clone = SsTable::load -> "
                                     "Checksums::verify) in one GPU batch per tick, beside the traffic",
                             "ticks": ticks, "failed": failed},
        "readback": {"keys": len(keys), "mismatches": mismatches,
                     "replayed_remove_reads_table_value": resurrected},
        "cpu_baseline": {"value": round(done / GIB / tc, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                         "sample": f"first {done / GIB:.2f} GiB of data+index files, oracle FIPS SHA-256, 1 thread"},
        "synthesis_s": synth["seconds"],
    }
    print(json.dumps(res), flush=True)
    if not a.keep:
        shutil.rmtree(a.dir, ignore_errors=True)
    if mismatches:
        sys.exit(1)


if __name__ == "__main__":
    main()
