"""Config 5 (end-to-end tree load verify): the synthetic tree is in the
reference's on-disk layout (checked against the oracle on CPU), and
load_verify() reproduces Db::load's checksum behaviour on the GPU (first bad
table panics naming its data / index file, a corrupted WAL Insert is
WalError::CorruptedData)."""
import json
import os
import struct

import pytest

from lsm_storage_engine_amd import _lib, tree
from lsm_storage_engine_amd.checksums import ChecksumPanic
from lsm_storage_engine_amd.sstable_metadata import SsTableMetadata
from lsm_storage_engine_amd.wal import CorruptedData
from oracle import oracle as O


@pytest.fixture(scope="module")
def small_tree(tmp_path_factory):
    base = str(tmp_path_factory.mktemp("tree"))
    info = tree.synthesize_tree(base, 6 << 20, wal_records=3000, threads=4)
    return base, info


def test_tree_layout_matches_oracle(small_tree):
    base, info = small_tree
    metas = tree.list_tables(base)
    assert len(metas) == info["tables"] and len(metas) >= tree.SSTABLE_MAX_LEVEL
    assert [m.level for m in metas] == sorted(m.level for m in metas)
    total = 0
    for m in metas:
        with open(m.checksum_path()) as f:
            cj = f.read()
        # checksums.rs:64-80 JSON, digests by the oracle (FIPS SHA-256 + base64 STANDARD)
        assert cj == O.checksums_json(O.file_checksum(m.index_path()), O.file_checksum(m.data_path()))
        data = open(m.data_path(), "rb").read()
        pos, n, keys = 0, 0, []
        while pos < len(data):  # datafile.rs:27-35 records fill the file exactly
            kl, vl = struct.unpack_from("<II", data, pos)
            keys.append((data[pos + 8:pos + 8 + kl], pos))
            pos += 8 + kl + vl
            n += 1
        assert pos == len(data)
        assert [k for k, _ in keys] == sorted(k for k, _ in keys)
        idx = open(m.index_path(), "rb").read()  # bincode BTreeMap<Vec<u8>, u64>
        cnt = struct.unpack_from("<Q", idx, 0)[0]
        assert cnt == (n + tree.INDEX_STEP - 1) // tree.INDEX_STEP
        p = 8
        for i in range(cnt):
            kl = struct.unpack_from("<Q", idx, p)[0]
            key = idx[p + 8:p + 8 + kl]
            off = struct.unpack_from("<Q", idx, p + 8 + kl)[0]
            assert (key, off) == keys[i * tree.INDEX_STEP]
            p += 16 + kl
        assert p == len(idx)
        meta = json.load(open(m.metadata_path()))
        assert list(meta) == ["base_path", "id", "level", "metadata_filename", "checksum_filename",
                              "data_filename", "index_filename", "bloom_filter_filename"]
        total += len(data) + len(idx)
    assert total == info["table_bytes"]
    st, recs, _ = O.wal_replay(open(os.path.join(base, "wal", "wal.log"), "rb").read())
    assert st == 0 and len(recs) == 3000


@pytest.mark.gpu
def test_load_verify_clean_and_corrupted(ctx, small_tree, tmp_path):
    import shutil
    base = str(tmp_path / "t")
    shutil.copytree(small_tree[0], base)
    for p in tree.scan_order(base):  # metadata base_path points at the original tree: rewrite it
        d = json.load(open(p))
        d["base_path"] = base
        with open(p, "w") as f:
            f.write(json.dumps(d, separators=(",", ":")))
    metas = tree.list_tables(base)
    assert all(m.base_path == base for m in metas)
    mem, rep = tree.load_verify(ctx, base)
    assert rep["tables"] == len(metas) and rep["wal_records"] == 3000
    _, recs, _ = O.wal_replay(open(os.path.join(base, "wal", "wal.log"), "rb").read())
    assert mem.size() <= 3000 and mem.size() > 0
    assert rep["table_bytes"] == small_tree[1]["table_bytes"]
    # lsmck_tree_verify_listed: the verify's own listing, in load order, as the metadata files say
    listed = []
    ctx.tree_verify(base, listed=listed)
    assert [e["metadata_path"] for e in listed] == tree.scan_order(base)
    for e in listed:
        m = SsTableMetadata.load(e["metadata_path"])
        assert e["status"] == 0 and (e["data_path"], e["index_path"], e["checksum_path"]) == (
            m.data_path(), m.index_path(), m.checksum_path())
        assert (int(e["id"]), e["level"]) == (m.id, m.level)
    # the second table (load order) has its index file corrupted: panic naming the index file
    paths = tree.scan_order(base)
    order = [SsTableMetadata.load(p) for p in paths]
    with open(order[1].index_path(), "r+b") as f:
        f.seek(9)
        f.write(b"\xff")
    with pytest.raises(ChecksumPanic, match=order[1].index_filename):
        tree.load_verify(ctx, base)
    r = ctx.tree_verify(base)
    assert (r["bad_tables"], r["first_index"], r["first_status"]) == (1, 1, 2)
    # ... and the first table's data file too: the first table in load order wins
    with open(order[0].data_path(), "r+b") as f:
        f.seek(100)
        f.write(b"\x00\x01\x02")
    with pytest.raises(ChecksumPanic, match=order[0].data_filename):
        tree.load_verify(ctx, base)
    r = ctx.tree_verify(base)
    assert (r["bad_tables"], r["first_index"], r["first_status"]) == (2, 0, 1)
    assert r["first_metadata_path"] == paths[0] == order[0].metadata_path()


@pytest.mark.gpu
def test_load_verify_corrupted_wal(ctx, tmp_path):
    base = str(tmp_path / "w")
    tree.synthesize_tree(base, 1 << 20, wal_records=500, threads=2)
    wal = os.path.join(base, "wal", "wal.log")
    img = bytearray(open(wal, "rb").read())
    st, recs, _ = O.wal_replay(bytes(img))
    ins = [r for r in recs if r.type == 1 and r.klen + r.vlen > 0]
    img[ins[10].payload_off] ^= 0x40  # flip a payload bit of the 11th non-empty Insert
    open(wal, "wb").write(bytes(img))
    with pytest.raises(CorruptedData):
        tree.load_verify(ctx, base)


# SsTableMetadata JSON as serde_json reads it (sstable_metadata.rs:7-17, 76-83):
# (text with BASE / TS substituted, the reference's outcome)
_F = ('"base_path":"BASE","id":TS,"level":0,"metadata_filename":"metadata_TS.db","checksum_filename":'
      '"checksum_TS.db","data_filename":"data_TS.db","index_filename":"index_TS.db","bloom_filter_filename":"bloom_TS.db"')
META_CASES = [
    ("{" + _F + "}", "ok"),
    (" {\n " + _F.replace(",", " ,\n\t") + " } \n", "ok"),                    # whitespace
    ('{"extra":[1,{"a":"}"}],' + _F + ',"z":null}', "ok"),                     # unknown fields ignored
    ("{" + _F.replace('"id":TS', '"id":340282366920938463463374607431768211455') + "}", "ok"),  # u128::MAX
    ("{" + _F.replace('"id":TS', '"id":340282366920938463463374607431768211456') + "}", "panic"),  # 2^128
    ("{" + _F.replace('"id":TS', '"id":1.5') + "}", "panic"),
    ("{" + _F.replace('"id":TS', '"id":-1') + "}", "panic"),
    ("{" + _F.replace('"id":TS', '"id":"TS"') + "}", "panic"),
    ("{" + _F.replace('"level":0', '"level":256') + "}", "panic"),
    ("{" + _F.replace('"level":0', '"level":00') + "}", "panic"),
    ("{" + _F.replace(',"bloom_filter_filename":"bloom_TS.db"', "") + "}", "panic"),  # missing field
    ("{" + _F + ',"level":0}', "panic"),                                       # duplicate field
    ("{" + _F + "}x", "panic"),                                                # trailing characters
    ("{" + _F.replace("data_TS.db", "da\\u0074a_TS.db") + "}", "ok"),        # escapes
    ("", "panic"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(META_CASES)))
def test_tree_verify_metadata_json(ctx, tmp_path, case):
    from lsm_storage_engine_amd import _lib, checksums
    text, want = META_CASES[case]
    base = str(tmp_path)
    m = SsTableMetadata.new(base, 0, timestamp_ms=1_700_000_000_123)
    os.makedirs(os.path.dirname(m.data_path()))
    open(m.data_path(), "wb").write(b"records" * 100)
    open(m.index_path(), "wb").write(b"index")
    checksums.Checksums.write_checksums(m)
    open(m.metadata_path(), "w").write(text.replace("BASE", base).replace("TS", str(m.id)))
    open(os.path.join(base, "level-0", "not-a-table.db"), "w").write("{}")  # name lacks "metadata": skipped
    listed = []
    r = ctx.tree_verify(base, listed=listed)
    assert r["tables"] == 1 and len(listed) == 1
    assert listed[0]["status"] == (0 if want == "ok" else _lib.META_PANIC)
    if want != "ok":
        assert listed[0]["id"] == listed[0]["data_path"] == ""
    if want == "ok":
        assert listed[0]["id"] == (str(m.id) if "340282" not in text else "340282366920938463463374607431768211455")
        assert listed[0]["data_path"] == m.data_path()  # escapes decoded
    assert all(os.path.isdir(os.path.join(base, f"level-{lv}")) for lv in range(5))  # create_dir_all
    if want == "ok":
        assert r["bad_tables"] == 0 and r["table_bytes"] == 705
    else:
        assert r["first_status"] == _lib.META_PANIC
        with pytest.raises(tree.MetadataPanic, match="unknown format"):
            tree.load_verify(ctx, base)


@pytest.mark.gpu
def test_tree_verify_empty_and_missing_files(ctx, tmp_path):
    base = str(tmp_path / "new")  # Db::load on a fresh path: creates the levels, no tables
    r = ctx.tree_verify(base)
    assert r["tables"] == 0 and r["bad_tables"] == 0
    m = SsTableMetadata.new(base, 2, timestamp_ms=1_700_000_000_999)
    m.write_to_file()  # a table whose data/index/checksum files are missing
    r = ctx.tree_verify(base)
    # the data file cannot be opened: calculate_checksum's panic (checksums.rs:25)
    assert r["tables"] == 1 and r["first_status"] == _lib.PANIC_OPEN_FILE
    with pytest.raises(ChecksumPanic, match="Can't open file to calculate checksum"):
        tree.load_verify(ctx, base)
    # data file present, index missing: the same panic on the index file
    open(m.data_path(), "wb").close()
    r = ctx.tree_verify(base)
    assert r["first_status"] == _lib.PANIC_OPEN_INDEX
    # both present, checksum file missing: "Can't open checksum file" (:46)
    open(m.index_path(), "wb").close()
    r = ctx.tree_verify(base)
    assert r["first_status"] == _lib.PANIC_OPEN_CHECKSUM
    with pytest.raises(ChecksumPanic, match="Can't open checksum file"):
        tree.load_verify(ctx, base)
    st = ctx.checksums_verify_many([(m.data_path(), m.index_path(), m.checksum_path()),
                                    (m.data_path() + "x", m.index_path(), m.checksum_path())])
    assert st == [_lib.PANIC_OPEN_CHECKSUM, _lib.PANIC_OPEN_FILE]


@pytest.mark.gpu
def test_tree_verify_large_files_on_host_threads(ctx, tmp_path):
    """Files at or above tree_cpu_file_bytes are hashed on host threads while
    the GPU streams the rest: same verdicts (clean, data mismatch, index
    mismatch, missing file) whichever side hashes a file."""
    base = str(tmp_path / "big")
    tree.synthesize_tree(base, 6 << 20, wal_records=10)
    metas = tree.list_tables(base)
    trip = [(m.data_path(), m.index_path(), m.checksum_path()) for m in metas]
    sizes = sorted(os.path.getsize(m.data_path()) for m in metas)
    try:
        for cut in (0, sizes[len(sizes) // 2], 1):  # default (all GPU), half and half, all on host threads
            ctx.set_option("tree_cpu_file_bytes", cut)
            assert ctx.checksums_verify_many(trip) == [0] * len(trip)
            big = max(range(len(metas)), key=lambda i: os.path.getsize(metas[i].data_path()))
            small = min(range(len(metas)), key=lambda i: os.path.getsize(metas[i].data_path()))
            saved = {}
            for i, which in ((big, 0), (small, 1)):
                p = trip[i][which]
                saved[p] = open(p, "rb").read()
                b = bytearray(saved[p])
                b[len(b) // 2] ^= 4
                open(p, "wb").write(bytes(b))
            st = ctx.checksums_verify_many(trip)
            assert st[big] == _lib.DATA_MISMATCH and st[small] == _lib.INDEX_MISMATCH
            assert sum(x != 0 for x in st) == 2
            for p, b in saved.items():
                open(p, "wb").write(b)
            os.rename(trip[big][0], trip[big][0] + ".gone")
            st = ctx.checksums_verify_many(trip)
            assert st[big] == _lib.PANIC_OPEN_FILE and sum(x != 0 for x in st) == 1
            os.rename(trip[big][0] + ".gone", trip[big][0])
    finally:
        ctx.set_option("tree_cpu_file_bytes", 0)


@pytest.mark.gpu
def test_multicontext_tree_verify(ctx, tmp_path):
    """lsmck_tree_verify_multi / lsmck_checksums_verify_many_multi: the tables
    split by bytes over three contexts (all on this box's one GPU; on a node,
    one per device and PCIe link) give the single-context verdicts."""
    from lsm_storage_engine_amd.device import MultiContext
    base = str(tmp_path / "multi")
    tree.synthesize_tree(base, 6 << 20, wal_records=200)
    mc = MultiContext(devices=[0, 0, 0])
    try:
        mem1, r1 = tree.load_verify(ctx, base)
        mem3, r3 = tree.load_verify(mc, base)
        assert mem1.data == mem3.data and r1["tables"] == r3["tables"] and r1["table_bytes"] == r3["table_bytes"]
        metas = tree.list_tables(base)
        trip = [(m.data_path(), m.index_path(), m.checksum_path()) for m in metas]
        for i, which in ((1, 0), (len(metas) // 2, 1), (len(metas) - 2, 0)):
            p = trip[i][which]
            b = bytearray(open(p, "rb").read())
            b[3] ^= 1
            open(p, "wb").write(bytes(b))
        assert mc.checksums_verify_many(trip) == ctx.checksums_verify_many(trip)
        assert sum(x != 0 for x in mc.checksums_verify_many(trip)) == 3
        a, b = ctx.tree_verify(base), mc.tree_verify(base)
        for k in ("tables", "table_bytes", "bad_tables", "first_index", "first_status", "first_metadata_path"):
            assert a[k] == b[k], k
    finally:
        for c in mc.ctxs:
            c.close()


@pytest.fixture(scope="module")
def tree_24mib(tmp_path_factory):
    base = str(tmp_path_factory.mktemp("tree24"))
    tree.synthesize_tree(base, 24 << 20, wal_records=1000, threads=4)
    return base


@pytest.mark.gpu
def test_tree_verify_top_level_beside_the_listing(ctx, tree_24mib, tmp_path):
    """"tree_overlap": the highest level's tables verified while the lower
    levels are listed (forced on this small tree) reports exactly what one
    batch does: the same listing, statuses and first failure in read_dir order
    (db.rs:37-59), with corruptions in either part."""
    import shutil
    base = str(tmp_path / "o")
    shutil.copytree(tree_24mib, base)
    for p in tree.scan_order(base):
        d = json.load(open(p))
        d["base_path"] = base
        with open(p, "w") as f:
            f.write(json.dumps(d, separators=(",", ":")))
    paths = tree.scan_order(base)
    order = [SsTableMetadata.load(p) for p in paths]
    top = max(m.level for m in order)
    assert sum(m.level == top for m in order) > 8  # (the two-part form has a second part)
    it = [i for i, m in enumerate(order) if m.level == top][-1]  # (in the second part when there is one)
    il = next(i for i, m in enumerate(order) if m.level == 1)
    keys = ("tables", "table_bytes", "bad_tables", "first_index", "first_status", "first_metadata_path")

    def both():
        out = []
        # one batch; the top level beside the listing in one part; in two (the
        # first 8 tables early, listing batches of 2 names)
        for v, lb in ((0, 0), (3, 0), (1, 2)):
            ctx.set_option("tree_overlap", v)
            ctx.set_option("tree_list_batch", lb)
            listed = []
            r = ctx.tree_verify(base, listed=listed)
            out.append(({k: r[k] for k in keys}, [(e["metadata_path"], e["status"]) for e in listed]))
        assert out[0] == out[1] == out[2]
        return out[0][0]

    try:
        r = both()
        assert r["bad_tables"] == 0 and r["tables"] == len(order)
        with open(order[it].data_path(), "r+b") as f:  # a top-level table: verified in the early batch
            f.seek(5)
            f.write(b"\x7f")
        r = both()
        assert (r["bad_tables"], r["first_index"], r["first_status"]) == (1, it, 1)
        with open(order[il].index_path(), "r+b") as f:  # a level-1 table: earlier in read_dir order
            f.seek(9)
            f.write(b"\xff")
        r = both()
        assert (r["bad_tables"], r["first_index"], r["first_status"]) == (2, il, 2)
        assert r["first_metadata_path"] == paths[il]
    finally:
        ctx.set_option("tree_overlap", 2048)
        ctx.set_option("tree_list_batch", 0)
