"""The checksum work of ``Db::load`` over a whole LSM tree (BASELINE config 5).

``Db::load`` (src/tokio/db.rs:37-73) walks ``<base>/level-0 .. level-4``
(SSTABLE_MAX_LEVEL = 5, db.rs:17), loads every table whose file name contains
"metadata" (db.rs:48-55) -- ``SsTable::load`` verifies the table's checksum file
first (src/tokio/sstable.rs:32-34 -> checksums.rs:40-62) -- and then replays
``<base>/wal/wal.log`` into the memtable (db.rs:60-63, memtable.rs:28-47).

``load_verify(ctx, base)`` does that checksum work as two GPU batches: every
data and index file of the tree through the streaming
``lsmck_checksums_verify_many`` (length-ordered SHA-256), and the WAL through
``lsmck_wal_replay_verify`` (CRC-32).  The first failing table in load order
raises ``ChecksumPanic`` with the reference's message, as its panic would.

``synthesize_tree`` writes a tree in the reference's on-disk layout (data file
datafile.rs:27-35, bincode index sstable_index.rs:42-46 with INDEX_STEP = 100,
checksum JSON checksums.rs:64-80, metadata JSON sstable_metadata.rs:79-85,
WAL framing wal.rs:165-196).  It is the fixture generator of the end-to-end
benchmark (tools/e2e_tree.py), not part of the verified path: its checksum
files come from hashlib (OpenSSL), an implementation independent of liblsmck.
"""
import base64
import concurrent.futures as cf
import hashlib
import json
import mmap
import os
import struct
import time
import zlib

import numpy as np

from . import _lib
from .checksums import ChecksumPanic, Checksums, _raise_for
from .sstable_metadata import SsTableMetadata
from .wal import CommandLog, MemTable

SSTABLE_MAX_LEVEL = 5  # src/tokio/db.rs:17
INDEX_STEP = 100       # src/tokio/sstable.rs:17
KEY_LEN = 16


def _b64sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return base64.b64encode(h.digest()).decode()


def _table_bytes(rng, first_key, target):
    """One table's data and index file contents: records
    [u32 klen][u32 vlen][key][val] (datafile.rs:27-35) in key order, keys
    b"%016d", values 100..4000 random bytes; the index maps every
    INDEX_STEP-th key to its offset (bincode: u64 count, then u64 len, key,
    u64 offset per entry)."""
    vlen = rng.integers(100, 4001, size=max(1, target // 2058 + 8)).astype(np.int64)
    rec = 8 + KEY_LEN + vlen
    end = np.cumsum(rec)
    m = int(np.searchsorted(end, target)) + 1
    m = min(m, len(vlen))
    vlen, rec = vlen[:m], rec[:m]
    pos = np.zeros(m, dtype=np.int64)
    pos[1:] = np.cumsum(rec[:-1])
    total = int(pos[-1] + rec[-1])
    buf = np.frombuffer(rng.bytes(total), dtype=np.uint8).copy()
    hdr = np.empty((m, 8), dtype=np.uint8)
    hdr[:, 0:4] = np.frombuffer(np.full(m, KEY_LEN, dtype="<u4").tobytes(), dtype=np.uint8).reshape(m, 4)
    hdr[:, 4:8] = np.frombuffer(vlen.astype("<u4").tobytes(), dtype=np.uint8).reshape(m, 4)
    nums = first_key + np.arange(m, dtype=np.int64)
    keys = ((nums[:, None] // (10 ** np.arange(KEY_LEN - 1, -1, -1, dtype=np.int64))[None, :]) % 10 + 48).astype(np.uint8)
    cols = pos[:, None] + np.arange(8)[None, :]
    buf[cols] = hdr
    cols = pos[:, None] + 8 + np.arange(KEY_LEN)[None, :]
    buf[cols] = keys
    idx = bytearray(struct.pack("<Q", (m + INDEX_STEP - 1) // INDEX_STEP))
    for i in range(0, m, INDEX_STEP):
        idx += struct.pack("<Q", KEY_LEN) + keys[i].tobytes() + struct.pack("<Q", int(pos[i]))
    return buf, bytes(idx), m


def synthesize_tree(base, data_bytes, seed=0x5EED0005, wal_records=200_000, threads=8, progress=None):
    """Write a tree of about ``data_bytes`` of SSTable data files under ``base``.
    Level i holds tables of about 4 KiB * 4^i: ~4 KiB level-0 tables (a flushed
    memtable at the reference's default config) up to ~1 MiB at level 4, which
    holds most of the bytes, as a compacted tree does (a
    100 GiB tree is ~10^5 files of <= ~1 MiB).  Returns a summary."""
    t0 = time.perf_counter()
    rng = np.random.default_rng(seed)
    share = [0.001, 0.004, 0.025, 0.12, 0.85]
    plan = []  # (level, target bytes)
    for lv in range(SSTABLE_MAX_LEVEL):
        tsize = 4096 << (2 * lv)
        left = int(data_bytes * share[lv])
        while left > 0:
            t = int(min(left, tsize * rng.uniform(0.75, 1.25)))
            plan.append((lv, max(t, 4096)))
            left -= t
    for lv in range(SSTABLE_MAX_LEVEL):
        os.makedirs(os.path.join(base, f"level-{lv}"), exist_ok=True)
    seeds = rng.integers(0, 2**63, size=len(plan))
    first = np.concatenate([[0], np.cumsum([p[1] // 2000 + 1 for p in plan])[:-1]])

    def write_one(i):
        lv, target = plan[i]
        r = np.random.default_rng(int(seeds[i]))
        m = SsTableMetadata.new(base, lv, timestamp_ms=1_700_000_000_000 + i)
        data, index, nrec = _table_bytes(r, int(first[i]) * 100, target)
        with open(m.data_path(), "wb") as f:
            f.write(memoryview(data))
        with open(m.index_path(), "wb") as f:
            f.write(index)
        with open(m.checksum_path(), "w") as f:
            f.write(json.dumps({"index_checksum": _b64sha(m.index_path()), "data_checksum": _b64sha(m.data_path())},
                               separators=(",", ":")))
        open(m.bloom_filter_path(), "wb").close()  # not checksummed; the load path here does not read it
        m.write_to_file()
        return len(data) + len(index)

    table_bytes = 0
    with cf.ThreadPoolExecutor(threads) as ex:
        for i, b in enumerate(ex.map(write_one, range(len(plan)))):
            table_bytes += b
            if progress and (i + 1) % 2048 == 0:
                progress(f"synthesize_tree: {i + 1}/{len(plan)} tables, {table_bytes / 2**30:.1f} GiB")
    # WAL: inserts and removes of random keys, framed as CommandLog::log
    os.makedirs(os.path.join(base, "wal"), exist_ok=True)
    wal = bytearray()
    pool = rng.bytes(1 << 20)
    kl = rng.integers(1, 40, size=wal_records)
    vl = rng.integers(0, 1000, size=wal_records)
    rm = rng.random(wal_records) < 0.1
    for i in range(wal_records):
        o = (i * 7919) % ((1 << 20) - 1100)
        key = pool[o:o + int(kl[i])]
        if rm[i]:
            wal += struct.pack("<BII", 2, zlib.crc32(key), len(key)) + key
        else:
            d = key + pool[o + 40:o + 40 + int(vl[i])]
            wal += struct.pack("<BIII", 1, zlib.crc32(d), len(key), int(vl[i])) + d
    with open(os.path.join(base, "wal", "wal.log"), "wb") as f:
        f.write(wal)
    return {"tables": len(plan), "table_bytes": table_bytes, "wal_bytes": len(wal), "wal_records": wal_records,
            "seconds": round(time.perf_counter() - t0, 2)}


def list_tables(base):
    """db.rs:40-58: per level, every file whose name contains "metadata"."""
    metas = []
    for lv in range(SSTABLE_MAX_LEVEL):
        d = os.path.join(base, f"level-{lv}")
        os.makedirs(d, exist_ok=True)
        level = [SsTableMetadata.load(os.path.join(d, n)) for n in os.listdir(d) if "metadata" in n]
        level.sort(key=lambda m: m.id)  # tables.sort() (SsTable orders by id)
        metas.extend(level)
    return metas


class MetadataPanic(RuntimeError):
    """SsTableMetadata::load's panic (sstable_metadata.rs:76-83)."""


def _raise_first(rep):
    st, mpath = rep["first_status"], rep["first_metadata_path"]
    if st == _lib.META_PANIC:
        if not os.access(mpath, os.R_OK):
            raise MetadataPanic("Can't open metadata file")
        raise MetadataPanic("Can't read metadata file, file with unknown format")
    _raise_for(st, SsTableMetadata.load(mpath))


def scan_order(base):
    """Metadata paths in Db::load's load order: level by level, read_dir order
    within a level (db.rs:40-55) -- the order in which the reference verifies
    tables and hence which failing table it panics on."""
    out = []
    for lv in range(SSTABLE_MAX_LEVEL):
        d = os.path.join(base, f"level-{lv}")
        out.extend(os.path.join(d, n) for n in os.listdir(d) if "metadata" in n)
    return out


def load_verify(ctx, base):
    """The checksum work of Db::load (db.rs:37-73) as two GPU batches.
    Returns (memtable, report); raises ChecksumPanic / MetadataPanic /
    WalError where the reference panics / errors.  The table scan (listing,
    metadata parsing, verify) is native: lsmck_tree_verify."""
    rep = ctx.tree_verify(base)
    if rep["first_status"] is not None:
        _raise_first(rep)
    nbytes = rep["table_bytes"]
    # WAL: CommandLog::new + MemTable::from_log (db.rs:60-63); the checksum work
    # is one lsmck_wal_replay_verify batch (timed alone), the BTreeMap build after it
    wal_path = os.path.join(base, "wal", "wal.log")
    log = CommandLog.new(wal_path)
    try:
        t3 = time.perf_counter()
        # the log is mapped, not read(): read() into a fresh bytes object costs
        # page faults plus a copy (0.15 s for 0.24 GB, more than the verify);
        # the host walk and the staged upload read the mapping in place
        n = os.fstat(log.file.fileno()).st_size
        mm = mmap.mmap(log.file.fileno(), n, access=mmap.ACCESS_READ) if n else None
        img = mm if mm is not None else b""
        records, wst, bad = ctx.wal_replay_verify(img)
        t4 = time.perf_counter()
        wal_bytes = len(img)
        if mm is not None:
            mm.close()
        log.file.seek(0)
        mem = MemTable.from_log(log, ctx)  # raises the reference's WalError / panic for a bad log
        t5 = time.perf_counter()
    finally:
        log.file.close()
    list_s, tables_s = rep["list_seconds"], rep["verify_seconds"]
    return mem, {"tables": rep["tables"], "table_bytes": nbytes, "wal_bytes": wal_bytes, "wal_records": len(records),
                 "list_s": list_s, "tables_s": tables_s, "wal_s": t4 - t3, "memtable_build_s": t5 - t4,
                 "total_s": list_s + tables_s + (t4 - t3),
                 "tables_split": {k: rep[k] for k in ("stat_seconds", "read_seconds", "gpu_wait_seconds",
                                                      "compare_seconds", "rounds", "fds_cached")}}


__all__ = ["synthesize_tree", "list_tables", "scan_order", "load_verify", "ChecksumPanic", "MetadataPanic", "SSTABLE_MAX_LEVEL"]
