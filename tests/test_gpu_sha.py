"""GPU parity for the batched SHA-256 (lsmck_sha256_batch / _fixed) and the
whole-tree SSTable verify (lsmck_checksums_verify_many), against FIPS vectors,
the golden slices, the oracle, and the reference's checksum-file semantics."""
import os
import shutil

import numpy as np
import pytest

from lsm_storage_engine_amd import _lib
from lsm_storage_engine_amd.checksums import Checksums
from lsm_storage_engine_amd.sstable_metadata import SsTableMetadata
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_fips_and_golden_slices(ctx, golden, blob):
    texts = [e["text"].encode() for e in golden["sha256_text"]]
    data = np.frombuffer(b"".join(texts), dtype=np.uint8)
    ln = np.array([len(t) for t in texts], dtype=np.uint32)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    got = ctx.sha256(data, off, ln)
    for i, e in enumerate(golden["sha256_text"]):
        assert got[i].tobytes().hex() == e["sha256"]
    B = np.frombuffer(blob, dtype=np.uint8)
    sl = golden["sha256_slices"]
    got = ctx.sha256(B, np.array([e["off"] for e in sl], np.uint64), np.array([e["len"] for e in sl], np.uint32))
    for i, e in enumerate(sl):
        assert got[i].tobytes().hex() == e["sha256"], e


@pytest.fixture(params=[0, 1, 3], ids=["win1", "win2", "lines"])
def sha_pair(request, ctx):
    """The SHA-256 load windows: one block (68 B) or two blocks (132 B) per
    load, or whole aligned 128-B lines realigned through LDS rows."""
    ctx.set_option("sha_pair", request.param)
    yield request.param
    ctx.set_option("sha_pair", 1)


@pytest.mark.parametrize("length,stride,shift", [(4096, 4096, 0), (64, 64, 0), (55, 57, 1), (56, 59, 2),
                                                 (1000, 1003, 3), (0, 8, 0), (100000, 100000, 0),
                                                 (191, 193, 1), (192, 196, 2), (255, 257, 3), (256, 256, 0)])
def test_fixed_vs_oracle(ctx, sha_pair, length, stride, shift):
    n = max(1, min(20000, (32 << 20) // max(stride, 1)))
    data = O.gen_stream(21, 0, n * stride + shift + 8)
    base = data[shift:]
    got = ctx.sha256_fixed(base, stride, length, n)
    off = np.arange(n, dtype=np.uint64) * stride
    want = O.sha256_batch(base, off, np.full(n, length, np.uint32), threads=8)
    assert np.array_equal(got, want)


def test_random_lengths_vs_oracle(ctx, sha_pair):
    rng = np.random.default_rng(4)
    n = 20000
    ln = rng.integers(0, 3000, n).astype(np.uint32)
    off = np.concatenate([[3], 3 + np.cumsum(ln)[:-1]]).astype(np.uint64)
    data = O.gen_stream(22, 0, int(off[-1]) + int(ln[-1]) + 8)
    assert np.array_equal(ctx.sha256(data, off, ln), O.sha256_batch(data, off, ln, threads=8))


def test_device_path_fixed_4k(ctx):
    n = 1 << 14
    d = ctx.alloc(n * 4096)
    ctx.gen_stream(d.ptr, 0x5EED0002, 0, n * 4096)
    out = ctx.alloc(32 * n)
    ctx.sha256_fixed_device(d.ptr, 4096, 4096, n, out.ptr)
    ctx.sync()
    host = O.gen_stream(0x5EED0002, 0, n * 4096)
    want = O.sha256_batch(host, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096, np.uint32), threads=8)
    assert np.array_equal(out.download(np.uint8).reshape(n, 32), want)


def test_verify_many_tree(ctx, tmp_path, golden):
    g = golden["sstable_test"]
    metas = []
    for t in range(40):
        m = SsTableMetadata.new(str(tmp_path), t % 5, timestamp_ms=1000 + t)
        os.makedirs(os.path.dirname(m.data_path()), exist_ok=True)
        data = open(os.path.join(GOLDEN, g["data"]), "rb").read() * (1 + t % 7)
        with open(m.data_path(), "wb") as f:
            f.write(data)
        shutil.copy(os.path.join(GOLDEN, g["index"]), m.index_path())
        Checksums.write_checksums(m)
        metas.append(m)
    assert Checksums.verify_many(ctx, metas) == [0] * 40
    with open(metas[3].data_path(), "r+b") as f:
        f.write(b"Z")
    with open(metas[7].index_path(), "r+b") as f:
        f.seek(50)
        f.write(b"Z")
    os.remove(metas[9].checksum_path())
    st = Checksums.verify_many(ctx, metas)
    assert st[3] == _lib.DATA_MISMATCH and st[7] == _lib.INDEX_MISMATCH
    assert st[9] == _lib.PANIC_OPEN_CHECKSUM  # verify's .expect("Can't open checksum file"), checksums.rs:46
    assert sum(1 for s in st if s) == 3


@pytest.mark.parametrize("active,slice_bytes,open_files", [(0, 0, -1), (7, 4096, -1), (64, 64, -1), (1, 1 << 20, -1),
                                                            (64, 4096, 10), (7, 4096, 0)])
def test_verify_many_streaming(ctx, tmp_path, active, slice_bytes, open_files):
    """The slice-streamed whole-tree verify (defaults: 8192 files in flight,
    64 KiB per round; then few files in flight and small slices, so files span
    many rounds, slots are reused, and one slice per round): 300 tables of
    0..300 KiB data files, empty files, a 3 MiB table, a missing data file, a
    missing checksum file and single-byte corruptions.  Checksum files are
    written by the oracle (FIPS SHA-256 + base64 + the checksums.rs JSON)."""
    rng = np.random.default_rng(11)
    metas = []
    for t in range(300):
        m = SsTableMetadata.new(str(tmp_path), t % 5, timestamp_ms=5000 + t)
        os.makedirs(os.path.dirname(m.data_path()), exist_ok=True)
        n = 0 if t % 37 == 0 else (3 << 20) + 7 if t == 150 else int(rng.integers(1, 300 << 10))
        with open(m.data_path(), "wb") as f:
            f.write(O.gen_stream(900 + t, 0, n).tobytes())
        with open(m.index_path(), "wb") as f:
            f.write(O.gen_stream(70000 + t, 0, int(rng.integers(0, 2000))).tobytes())
        with open(m.checksum_path(), "w") as f:
            f.write(O.checksums_json(O.file_checksum(m.index_path()), O.file_checksum(m.data_path())))
        metas.append(m)
    ctx.set_option("tree_active_files", active)
    ctx.set_option("tree_slice_bytes", slice_bytes)
    ctx.set_option("tree_open_files", open_files)  # files kept open between slices; the rest reopen
    try:
        assert Checksums.verify_many(ctx, metas) == [0] * 300
        with open(metas[150].data_path(), "r+b") as f:  # the large table, last byte
            f.seek((3 << 20) + 6)
            f.write(b"\x00" if f.read(1) != b"\x00" else b"\x01")
        with open(metas[201].index_path(), "ab") as f:
            f.write(b"+")
        os.remove(metas[77].data_path())
        os.remove(metas[78].checksum_path())
        st = Checksums.verify_many(ctx, metas)
    finally:
        ctx.set_option("tree_active_files", 0)
        ctx.set_option("tree_slice_bytes", 0)
        ctx.set_option("tree_open_files", -1)
    assert st[150] == _lib.DATA_MISMATCH and st[201] == _lib.INDEX_MISMATCH
    assert st[77] == _lib.PANIC_OPEN_FILE  # calculate_checksum's .expect on the data file, checksums.rs:25
    assert st[78] == _lib.PANIC_OPEN_CHECKSUM  # checksums.rs:46
    assert sum(1 for s in st if s) == 4


@pytest.mark.parametrize("order,shift,start", [(1, 2, 128), (1, 0, 128), (1, 3, 16), (0, 2, 128)])
def test_length_sorted_batch(ctx, order, shift, start):
    """Variable-length batches of >= 2048 messages run in decreasing length
    order (lsmck_order.hip, "sha_order" 1) -- or batch order (0): the digests
    land at each message's own index either way.  Zipf lengths (config 3's
    shape) plus empty, 55/56/63/64-byte (padding edges) and > 64 KiB messages,
    scattered and unsorted."""
    rng = np.random.default_rng(77)
    n = 6000
    ln = O.gen_zipf_lengths(0x5EED0003, n).astype(np.uint32)
    ln[:8] = [0, 1, 55, 56, 63, 64, 65, 119]
    ln[8:12] = [70000, 131072, 200001, 65536]  # the log-spaced buckets
    ln[12:16] = [127 * 64, 128 * 64 - 9, 1023 * 64 - 10, 1024 * 64 - 9]  # edges of the coarse buckets
    ln = ln[rng.permutation(n)]
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + rng.integers(0, 5, n - 1).astype(np.uint64))
    total = int(off[-1]) + int(ln[-1])
    data = O.gen_stream(0x5EED0031, 0, total + 8)
    ctx.set_option("sha_order", order)
    ctx.set_option("sha_bucket_shift", shift)
    ctx.set_option("sha_bucket_from", start)
    try:
        got = ctx.sha256(data, off, ln)
    finally:
        ctx.set_option("sha_order", 1)
        ctx.set_option("sha_bucket_shift", 2)
        ctx.set_option("sha_bucket_from", 128)
    assert np.array_equal(got, O.sha256_batch(data, off, ln, threads=8))


@pytest.mark.parametrize("short", [0, 1, 3, 8, 12, 127])
def test_short_tail_on_the_lean_kernel(ctx, short):
    """"sha_short_blocks" N: in a length-ordered batch, the messages of at most
    N compression blocks (the order's tail, found on the device) run on the
    lean kernel, the rest on the window kernel; every digest at its message's
    index, identical to the oracle.  Host and device batches."""
    rng = np.random.default_rng(78 + short)
    n = 5000
    ln = O.gen_zipf_lengths(0x5EED0033, n).astype(np.uint32)
    ln[:10] = [0, 1, 55, 56, 63, 64, 119, 120, 183, 184]  # 1 / 2 / 3 / 4 blocks at the edges
    ln = ln[rng.permutation(n)]
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + rng.integers(0, 5, n - 1).astype(np.uint64))
    total = int(off[-1]) + int(ln[-1])
    data = O.gen_stream(0x5EED0034, 0, total + 8)
    want = O.sha256_batch(data, off, ln, threads=8)
    ctx.set_option("sha_short_blocks", short)
    try:
        assert np.array_equal(ctx.sha256(data, off, ln), want)
        d, d_o, d_l, out = ctx.alloc(total + 8), ctx.alloc(8 * n), ctx.alloc(4 * n), ctx.alloc(32 * n)
        try:
            d.upload(data)
            d_o.upload(off)
            d_l.upload(ln)
            ctx.sha256_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
            ctx.sync()
            assert np.array_equal(out.download(np.uint8).reshape(n, 32), want)
        finally:
            for b in (d, d_o, d_l, out):
                b.free()
    finally:
        ctx.set_option("sha_short_blocks", 12)


def _summaries():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "summaries.json")) as f:
        return json.load(f)


def test_config2_full_size_summary(ctx):
    """SHA-256 of all 2^24 4 KiB blocks of BASELINE config 2 (64 GiB,
    device-resident): CRC-32 of the 512 MiB digest array equals the oracle's
    (tests/golden/make_summaries.py)."""
    import zlib
    n = 1 << 24
    d = ctx.alloc(n * 4096)
    ctx.gen_stream(d.ptr, 0x5EED0002, 0, n * 4096)
    out = ctx.alloc(32 * n)
    ctx.sha256_fixed_device(d.ptr, 4096, 4096, n, out.ptr)
    ctx.sync()
    assert "%08x" % zlib.crc32(out.download(np.uint8).tobytes()) == _summaries()["config2"]["summary_sha256"]
    d.free()
    out.free()


def test_config3_full_size_summary(ctx):
    """SHA-256 of all 2^26 Zipf records of BASELINE config 3 (~97 GiB packed,
    device-resident, length-ordered dispatch): digest-array CRC equals the oracle's."""
    import zlib
    from lsm_storage_engine_amd.device import gen_zipf_lengths
    n = 1 << 26
    ln = gen_zipf_lengths(0x5EED0003, n)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1].astype(np.uint64), out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    d = ctx.alloc(total + 64)
    ctx.gen_stream(d.ptr, 0x5EED0003, 0, total)
    d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(32 * n)
    d_o.upload(off)
    d_l.upload(ln)
    ctx.sha256_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
    ctx.sync()
    assert "%08x" % zlib.crc32(out.download(np.uint8).tobytes()) == _summaries()["config3"]["summary_sha256"]
    for buf in (d, d_o, d_l, out):
        buf.free()
