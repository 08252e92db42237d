"""GPU parity for the batched CRC-32 (lsmck_crc32_batch / _fixed / _verify):
bit-exact against the oracle (crc 1.x restatement) and the golden vectors,
over the edge cases of the reference's domain: empty and 1..3-byte records,
every first-segment length, unaligned starts, records packed back to back
(WAL-like) and scattered, segment-count boundaries of the combination tables
(>= 2^16 segments), and, at BASELINE sizes, size-independent properties."""
import numpy as np
import pytest

from lsm_storage_engine_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_golden_slices_host_path(ctx, golden, blob):
    B = np.frombuffer(blob, dtype=np.uint8)
    off = np.array([e["off"] for e in golden["crc32_slices"]], dtype=np.uint64)
    ln = np.array([e["len"] for e in golden["crc32_slices"]], dtype=np.uint32)
    want = np.array([e["crc"] for e in golden["crc32_slices"]], dtype=np.uint32)
    assert np.array_equal(ctx.crc32(B, off, ln), want)


def test_golden_slices_device_path(ctx, golden, blob):
    B = np.frombuffer(blob, dtype=np.uint8)
    sl = golden["crc32_slices"]
    off = np.array([e["off"] for e in sl], dtype=np.uint64)
    ln = np.array([e["len"] for e in sl], dtype=np.uint32)
    want = np.array([e["crc"] for e in sl], dtype=np.uint32)
    d_b, d_o, d_l, d_out = ctx.alloc(len(B)), ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * len(sl))
    d_b.upload(B)
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d_b.ptr, d_o.ptr, d_l.ptr, len(sl), d_out.ptr)
    ctx.sync()
    assert np.array_equal(d_out.download(np.uint32), want)
    # verify entry point: corrupt two expectations
    exp = want.copy()
    exp[[17, 900]] ^= 1
    d_e = ctx.alloc(exp.nbytes)
    d_e.upload(exp)
    rc, nbad, first = ctx.crc32_verify_device(d_b.ptr, d_o.ptr, d_l.ptr, d_e.ptr, len(sl))
    assert (rc, nbad, first) == (1, 2, 17)
    rc, nbad, first = ctx.crc32_verify(B, off, ln, want)
    assert (rc, nbad, first) == (0, 0, len(sl))


@pytest.mark.parametrize("length,stride,shift", [
    (256, 256, 0), (4096, 4096, 0), (128, 128, 0), (1, 1, 0), (3, 5, 1), (127, 131, 2), (129, 129, 3),
    (200, 208, 0), (4097, 4100, 4), (384, 400, 0), (65536, 65536, 0), (100000, 100003, 1), (0, 16, 0)])
def test_fixed_vs_oracle(ctx, length, stride, shift):
    n = max(1, min(40000, (64 << 20) // max(stride, 1)))
    data = O.gen_stream(0x5EED0002, 0, n * stride + shift + 16)
    base = data[shift:]
    got = ctx.crc32_fixed(base, stride, length, n)
    want = O.crc32_fixed(base, stride, length, n, threads=8)
    assert np.array_equal(got, want)


def _packed(lengths, gap_rng=None, align_shift=0):
    off = np.zeros(len(lengths), dtype=np.uint64)
    pos = align_shift
    for i, l in enumerate(lengths):
        if gap_rng is not None:
            pos += int(gap_rng.integers(0, 37))
        off[i] = pos
        pos += int(l)
    return off, pos


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_desc_random_vs_oracle(ctx, seed):
    rng = np.random.default_rng(seed)
    n = 30000
    kind = rng.integers(0, 4, n)
    ln = np.where(kind == 0, rng.integers(0, 8, n),
                  np.where(kind == 1, rng.integers(0, 300, n),
                           np.where(kind == 2, rng.integers(100, 5000, n), rng.integers(0, 70000, n)))).astype(np.uint32)
    off, total = _packed(ln, gap_rng=rng if seed != 2 else None, align_shift=seed)
    data = O.gen_stream(0x5EED0003 + seed, 0, total + 8)
    got = ctx.crc32(data, off, ln)
    want = O.crc32_batch(data, off, ln, threads=8)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (bad[:10], ln[bad[:10]], off[bad[:10]])


def test_desc_every_first_segment_length(ctx):
    # all record lengths 0..1030 (every first-segment length, 0-8 segments) at 4 alignments
    ln = np.tile(np.arange(0, 1031, dtype=np.uint32), 4)
    off, total = _packed(ln)
    off = off + np.repeat(np.arange(4, dtype=np.uint64), 1031)
    data = O.gen_stream(7, 0, total + 16)
    assert np.array_equal(ctx.crc32(data, off, ln), O.crc32_batch(data, off, ln, threads=8))


def test_desc_scattered_unsorted(ctx):
    rng = np.random.default_rng(9)
    data = O.gen_stream(11, 0, 8 << 20)
    n = 20000
    ln = rng.integers(0, 3000, n).astype(np.uint32)
    off = rng.integers(0, (8 << 20) - 3000, n).astype(np.uint64)  # overlapping, any order
    assert np.array_equal(ctx.crc32(data, off, ln), O.crc32_batch(data, off, ln, threads=8))


def test_large_records_high_segment_counts(ctx):
    # > 2^16 segments per record exercises the x^(8*128*65536*k) table
    ln = np.array([9 << 20, 3, (16 << 20) + 77, 4096, 0, 65537], dtype=np.uint32)
    off, total = _packed(ln, align_shift=1)
    data = O.gen_stream(12, 0, total + 8)
    assert np.array_equal(ctx.crc32(data, off, ln), O.crc32_batch(data, off, ln))


def test_zipf_config3_sample(ctx):
    n = 1 << 16
    ln = O.gen_zipf_lengths(0x5EED0003, n)
    off, total = _packed(ln)
    data = O.gen_stream(0x5EED0003, 0, total)
    assert np.array_equal(ctx.crc32(data, off, ln), O.crc32_batch(data, off, ln, threads=8))


def test_device_generated_fixed_4k(ctx):
    n = 1 << 15
    nbytes = n * 4096
    d = ctx.alloc(nbytes)
    ctx.gen_stream(d.ptr, 0x5EED0002, 0, nbytes)
    out = ctx.alloc(4 * n)
    ctx.crc32_fixed_device(d.ptr, 4096, 4096, n, out.ptr)
    ctx.sync()
    host = O.gen_stream(0x5EED0002, 0, nbytes)
    assert np.array_equal(d.download(np.uint8, count=4096 * 64), host[:4096 * 64])
    assert np.array_equal(out.download(np.uint32), O.crc32_fixed(host, 4096, 4096, n, threads=8))


@pytest.mark.parametrize("length,n", [(4096, (1 << 15) + 37), (256, (1 << 18) + 5), (128, 5000), (8192, 3)])
def test_fixed_ring_tiles(ctx, length, n):
    """Fixed records whose segment count divides 64 run the whole-tile ring
    kernel: several tiles per wave with a remainder, and batches where most
    waves have no tile."""
    nbytes = n * length
    d = ctx.alloc(nbytes)
    ctx.gen_stream(d.ptr, 0x5EED0020 + length, 0, nbytes)
    out = ctx.alloc(4 * n)
    ctx.crc32_fixed_device(d.ptr, length, length, n, out.ptr)
    ctx.sync()
    host = O.gen_stream(0x5EED0020 + length, 0, nbytes)
    assert np.array_equal(out.download(np.uint32), O.crc32_fixed(host, length, length, n, threads=8))
    d.free()
    out.free()


def _summaries():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "summaries.json")) as f:
        return json.load(f)


def test_config2_full_size_properties(ctx):
    """BASELINE config 2 at full size (2^24 x 4 KiB = 64 GiB, device-resident):
    (1) the fixed-record kernel and the descriptor path (different code
        paths: implicit offsets vs the stream kernel over off/len) agree on
        every record;
    (2) a sample of 4096 records spread over the whole buffer matches the oracle."""
    n = 1 << 24
    nbytes = n * 4096
    d = ctx.alloc(nbytes)
    ctx.gen_stream(d.ptr, 0x5EED0002, 0, nbytes)
    out_f = ctx.alloc(4 * n)
    ctx.crc32_fixed_device(d.ptr, 4096, 4096, n, out_f.ptr)
    off = (np.arange(n, dtype=np.uint64) * 4096)
    ln = np.full(n, 4096, dtype=np.uint32)
    d_o, d_l, out_d = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * n)
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out_d.ptr)
    ctx.sync()
    a, b = out_f.download(np.uint32), out_d.download(np.uint32)
    assert np.array_equal(a, b)
    # (3) the summary digest of all 2^24 CRCs equals the oracle's (tests/golden/make_summaries.py)
    import zlib
    assert "%08x" % zlib.crc32(a.astype("<u4").tobytes()) == _summaries()["config2"]["summary_crc32"]
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(n, 4096, replace=False))
    for i in idx[:4096]:
        assert a[i] == O.crc32(O.gen_stream(0x5EED0002, int(i) * 4096, 4096)), i
    for buf in (d, out_f, d_o, d_l, out_d):
        buf.free()


def test_fixed_kernel_paths_agree(ctx):
    """Every fixed-record path is bit-exact: the ring kernel (dword-aligned,
    segment count dividing 64), the two-slot kernel with per-lane columns
    (a stride too wide for one buffer window), whole segments whose count does
    not divide 64 (records straddle tiles), and unaligned records."""
    rng = np.random.default_rng(100)
    n = 6000
    ln = rng.integers(0, 9000, n).astype(np.uint32)
    ln[:5] = [0, 1, 3, 128, 129]
    off, total = _packed(ln, gap_rng=rng, align_shift=2)
    data = O.gen_stream(42, 0, total + 8)
    got = ctx.crc32(data, off, ln)
    fixed = ctx.crc32_fixed(data, 4096, 4096, total // 4096)
    small = ctx.crc32_fixed(data, 256, 256, total // 256)
    odd = ctx.crc32_fixed(data[1:], 300, 297, (total - 8) // 300)
    three = ctx.crc32_fixed(data[4:], 388, 384, (total - 8) // 388)
    assert np.array_equal(three, O.crc32_fixed(data[4:], 388, 384, (total - 8) // 388, threads=8))
    assert np.array_equal(small, O.crc32_fixed(data, 256, 256, total // 256, threads=8))
    assert np.array_equal(got, O.crc32_batch(data, off, ln, threads=8))
    assert np.array_equal(fixed, O.crc32_fixed(data, 4096, 4096, total // 4096, threads=8))
    assert np.array_equal(odd, O.crc32_fixed(data[1:], 300, 297, (total - 8) // 300, threads=8))
    # device records a stride beyond one buffer window apart (2^31 / 65): the
    # two-slot kernel with per-lane columns (host batches would be gathered)
    stride, nb = 40 << 20, 4
    d = ctx.alloc(stride * (nb - 1) + 4096)
    out = ctx.alloc(4 * nb)
    try:
        ctx.gen_stream(d.ptr, 43, 0, stride * (nb - 1) + 4096)
        ctx.crc32_fixed_device(d.ptr, stride, 4096, nb, out.ptr)
        ctx.sync()
        host = O.gen_stream(43, 0, stride * (nb - 1) + 4096)
        assert np.array_equal(out.download(np.uint32), O.crc32_fixed(host, stride, 4096, nb))
    finally:
        d.free()
        out.free()


def _device_crc(ctx, data, off, ln):
    d_b, d_o, d_l, d_out = ctx.alloc(len(data)), ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * len(off))
    d_b.upload(data)
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d_b.ptr, d_o.ptr, d_l.ptr, len(off), d_out.ptr)
    ctx.sync()
    return d_out.download(np.uint32)


def test_desc_records_just_after_page_boundary(ctx):
    """Record starts 0..15 bytes after a 4 KiB boundary of a (page-aligned) device
    buffer, every first-segment length: the group holding the record's first
    dword straddles the boundary, so it is loaded from the 16-byte aligned block
    at the boundary and shifted into place (seg_issue "risky" lanes)."""
    data = O.gen_stream(0x5EED0010, 0, 1 << 20)
    pages = np.arange(1, 200, dtype=np.uint64)
    d = np.arange(0, 16, dtype=np.uint64)
    lens = np.array([1, 2, 3, 4, 5, 7, 8, 12, 13, 16, 17, 100, 115, 116, 117, 127, 128, 129, 131, 140,
                     244, 255, 256, 257, 1000], dtype=np.uint32)
    P, D, L = np.meshgrid(pages, d, lens, indexing="ij")
    off = (P * 4096 + D).ravel().astype(np.uint64)
    ln = L.ravel().astype(np.uint32)
    got = _device_crc(ctx, data, off, ln)
    want = O.crc32_batch(data, off, ln, threads=8)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (bad[:10], off[bad[:10]], ln[bad[:10]])


def test_desc_records_at_allocation_edges(ctx):
    """Short records at offset 0 and flush with the end of the allocation
    (pad lanes of the last tile read nothing beyond the last record)."""
    n = 8192 + 37
    data = O.gen_stream(0x5EED0011, 0, n)
    for L in (1, 3, 5, 64, 127, 128, 129, 300):
        off = np.array([0, n - L, 1, n - L - 1], dtype=np.uint64)
        ln = np.full(4, L, dtype=np.uint32)
        assert np.array_equal(_device_crc(ctx, data, off, ln), O.crc32_batch(data, off, ln)), L


def test_config1_full_size(ctx):
    """BASELINE config 1 at full size on the GPU (2^20 x 256 B, device
    resident): every CRC equals the oracle's, and the summary digest (CRC-32 of
    the output array) is the pinned value of tests/test_oracle.py."""
    import zlib
    CONFIG1_SUMMARY_CRC32 = 0x727D43C0  # tests/test_oracle.py (oracle == zlib at config 1)
    assert "%08x" % CONFIG1_SUMMARY_CRC32 == _summaries()["config1"]["summary_crc32"]
    n = 1 << 20
    d = ctx.alloc(n * 256)
    ctx.gen_stream(d.ptr, 0x5EED0001, 0, n * 256)
    out = ctx.alloc(4 * n)
    ctx.crc32_fixed_device(d.ptr, 256, 256, n, out.ptr)
    ctx.sync()
    got = out.download(np.uint32)
    want = O.crc32_fixed(O.gen_stream(0x5EED0001, 0, n * 256), 256, 256, n, threads=8)
    assert np.array_equal(got, want)
    assert zlib.crc32(got.astype("<u4").tobytes()) == CONFIG1_SUMMARY_CRC32
    d.free()
    out.free()


def test_config3_full_size_summary(ctx):
    """BASELINE config 3 at full size (2^26 Zipf records, ~97 GiB packed,
    device-resident): the CRC-32 of the whole output array equals the oracle's
    (tests/golden/make_summaries.py), i.e. all 2^26 CRCs match."""
    import zlib
    from lsm_storage_engine_amd.device import gen_zipf_lengths
    n = 1 << 26
    ln = gen_zipf_lengths(0x5EED0003, n)
    assert np.array_equal(ln[:4096], O.gen_zipf_lengths(0x5EED0003, 4096))
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1].astype(np.uint64), out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    assert total == _summaries()["config3"]["payload_bytes"]
    d = ctx.alloc(total + 64)
    ctx.gen_stream(d.ptr, 0x5EED0003, 0, total)
    d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * n)
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
    ctx.sync()
    got = out.download(np.uint32)
    assert "%08x" % zlib.crc32(got.astype("<u4").tobytes()) == _summaries()["config3"]["summary_crc32"]
    for buf in (d, d_o, d_l, out):
        buf.free()


def test_config3w_full_size_summary(ctx):
    """Config 3's 2^26 records framed as wal.rs Insert records (a 13-byte header
    before every payload, ~98 GiB image, device-resident) through the caller
    entry point: the stream kernel takes the gapped batch, and the CRC-32 of
    the whole output array equals the oracle's (make_summaries.py config3w).
    Then the headers are written in front of the payloads (type 1, those CRCs,
    klen = min(len, 16)) and the 97.8 GiB log is replayed on the GPU: the
    segment walk of the headers (lsmck_segwalk.h, one pass over the whole log),
    every record found at its offset, every stored CRC checked, the records'
    CRC summary again the oracle's; then once more with compact records.""" 
    import zlib
    from lsm_storage_engine_amd.device import gen_zipf_lengths
    g = _summaries()["config3w"]
    n = 1 << 26
    ln = gen_zipf_lengths(0x5EED0003, n)
    off = np.full(n, 13, dtype=np.uint64)  # payload i+1 starts len[i] + 13 after payload i
    off[1:] += ln[:-1].astype(np.uint64)
    off = np.cumsum(off, dtype=np.uint64)
    total = int(off[-1]) + int(ln[-1])
    assert total == g["image_bytes"]
    d = ctx.alloc(total + 64)
    d_o, d_l, out = ctx.alloc(off.nbytes), ctx.alloc(ln.nbytes), ctx.alloc(4 * n)
    try:
        ctx.gen_stream(d.ptr, 0x5EED0003, 0, total)
        d_o.upload(off)
        d_l.upload(ln)
        ctx.set_option("crc_stream", 2)  # the stream kernel alone: a declined batch would leave outputs unwritten
        try:
            ctx.crc32_device(d.ptr, d_o.ptr, d_l.ptr, n, out.ptr)
            ctx.sync()
        finally:
            ctx.set_option("crc_stream", 1)
        got = out.download(np.uint32)
        assert "%08x" % zlib.crc32(got.astype("<u4").tobytes()) == g["summary_crc32"]
        # the same image as a WAL: headers in front of the payloads, then the replay
        ctx.wal_frame_insert_device(d.ptr, d_o.ptr, d_l.ptr, out.ptr, n, 16)
        ctx.sync()
        d_l.free()
        out.free()
        recs, st, bad = ctx.wal_replay_verify(total, device_ptr=d.ptr, cap=n)
        assert st == 0, bad
        assert len(recs) == n
        assert np.array_equal(recs.payload_off, off)
        assert np.array_equal(recs.rec_off, off - np.uint64(13))
        assert np.array_equal(recs.klen.astype(np.uint64) + recs.vlen, ln.astype(np.uint64))
        assert "%08x" % zlib.crc32(np.ascontiguousarray(recs.crc).astype("<u4").tobytes()) == g["summary_crc32"]
        del recs
        # the compact records (lsmck_wal_replay_verify16) into a page-locked
        # array by the SDMA read-back: every record at its offset, an Insert
        recs, st, bad = ctx.wal_replay_verify(total, device_ptr=d.ptr, cap=n, pinned_recs=True, compact=True)
        assert st == 0, bad
        assert len(recs) == n and recs.dtype.itemsize == 16
        assert np.array_equal(recs.payload_type, off)  # (bit 63 clear: Insert)
        assert np.array_equal(recs.klen.astype(np.uint64) + recs.vlen, ln.astype(np.uint64))
        del recs
    finally:
        for buf in (d, d_o, d_l, out):
            buf.free()


def test_multicontext_host_batches():
    """MultiContext: host batches split by bytes (variable) / count (fixed)
    over several contexts, each on its own host thread (here 3 contexts on
    device 0: the box has one GPU), identical to the oracle."""
    from lsm_storage_engine_amd.device import Context, MultiContext
    mc = MultiContext(contexts=[Context(0) for _ in range(3)])
    ln = O.gen_zipf_lengths(0x5EED0040, 20000)
    off, total = _packed(ln, align_shift=1)
    data = O.gen_stream(0x5EED0041, 0, total + 8)
    assert np.array_equal(mc.crc32(data, off, ln), O.crc32_batch(data, off, ln, threads=8))
    assert np.array_equal(mc.sha256(data, off, ln), np.asarray(O.sha256_batch(data, off, ln, threads=8)).reshape(-1, 32))
    n = 5001
    blk = O.gen_stream(0x5EED0042, 0, n * 300)
    assert np.array_equal(mc.crc32_fixed(blk, 300, 297, n), O.crc32_fixed(blk, 300, 297, n, threads=8))
    want = np.asarray(O.sha256_batch(blk, np.arange(n, dtype=np.uint64) * 300, np.full(n, 297, np.uint32),
                                     threads=8)).reshape(-1, 32)
    assert np.array_equal(mc.sha256_fixed(blk, 300, 297, n), want)
    assert len(mc.crc32(data, off[:2], ln[:2])) == 2  # fewer records than devices


from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None)
@given(st.lists(st.binary(max_size=1500), min_size=1, max_size=300), st.integers(0, 7), st.booleans())
def test_property_gpu_batches_vs_stdlib(ctx, recs, shift, packed):
    """Arbitrary record sets (empty records, any lengths and alignments,
    packed or with gaps) through the GPU batch paths against zlib.crc32 and
    hashlib.sha256: independent implementations of crc 1.x and sha2 0.10."""
    import hashlib
    import zlib
    gap = b"" if packed else b"\xa5" * 3
    buf = bytearray(b"\x00" * shift)
    off = []
    for r in recs:
        off.append(len(buf))
        buf += r + gap
    data = np.frombuffer(bytes(buf) + b"\0" * 8, dtype=np.uint8)
    off = np.array(off, dtype=np.uint64)
    ln = np.array([len(r) for r in recs], dtype=np.uint32)
    assert list(ctx.crc32(data, off, ln)) == [zlib.crc32(r) for r in recs]
    assert [bytes(d) for d in ctx.sha256(data, off, ln)] == [hashlib.sha256(r).digest() for r in recs]


def test_empty_batches_every_entry_point(ctx):
    """n = 0 everywhere: every batch entry point returns an empty result
    without a launch (and without touching the null or dangling pointers an
    empty Rust slice may carry)."""
    data = np.zeros(16, dtype=np.uint8)
    e64, e32 = np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint32)
    assert len(ctx.crc32(data, e64, e32)) == 0
    assert len(ctx.crc32_fixed(data, 16, 16, 0)) == 0
    assert len(ctx.sha256(data, e64, e32)) == 0
    assert len(ctx.sha256_fixed(data, 16, 16, 0)) == 0
    assert ctx.checksums_verify_many([]) == []
    recs, rc, _ = ctx.wal_replay_verify(b"")
    assert rc == 0 and len(recs) == 0
    d = ctx.alloc(64)
    out = ctx.alloc(64)
    ctx.crc32_fixed_device(d.ptr, 16, 16, 0, out.ptr)
    ctx.sha256_fixed_device(d.ptr, 16, 16, 0, out.ptr)
    ctx.sync()


def test_stage_numa_host_batches():
    """Staging placement (stage_numa): the device's node in effect by default
    on a multi-node host (none on a single-node one), every node and "off"
    accepted, a host batch's CRCs the oracle's under each -- pageable
    (staged on the pool's threads) and pinned (lsmck_host_alloc_pinned,
    allocated under the placement); out-of-range values refused."""
    import os
    from lsm_storage_engine_amd.device import Context
    nodes = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit()])
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, size=(20 << 20) + 777, dtype=np.uint8)
    off = np.sort(rng.integers(0, len(data) - 5000, size=3000)).astype(np.uint64)
    ln = rng.integers(0, 5000, size=3000).astype(np.uint32)
    want = np.array([O.crc32(data[int(o):int(o) + int(n)].tobytes()) for o, n in zip(off, ln)], dtype=np.uint32)
    for mode in [-2, -1] + list(range(nodes)):
        ctx = Context(0)
        try:
            dev_node = ctx.get_stat("numa_node")
            ctx.set_option("stage_numa", mode)
            eff = ctx.get_stat("stage_numa_node")
            if mode == -2:
                assert eff == (dev_node if nodes > 1 else -1)
            else:
                assert eff == mode
            assert (ctx.crc32(data, off, ln) == want).all()
            pb = ctx.alloc_pinned(len(data))
            pb.array[:] = data
            assert (ctx.crc32(pb.array, off, ln, pinned=True) == want).all()
            pb.free()
            with pytest.raises(_lib.LsmckError):
                ctx.set_option("stage_numa", -3)
        finally:
            ctx.close()
