"""The stream kernel (crc32_stream_kernel, lsmck_crc32.hip): sorted batches of
records -- packed back to back, or with gaps between them like the payloads of
a WAL image (wal.rs:165-196: a 13- or 9-byte header before each payload) --
checksummed from aligned 128-byte chunks of the byte stream, record starts as
CRC register resets and record ends as captures; records under 64 bytes by
their window lane.  Every case is checked against the oracle (crc 1.x's
algorithm, oracle/lsmck_oracle.c) and against the walking kernel on the same
records (crc_stream 0).  tools/stream_sim.py is the CPU model of the same
algebra."""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _packed(lens, lead):
    lens = np.asarray(lens, dtype=np.uint32)
    off = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        np.cumsum(lens[:-1].astype(np.uint64), out=off[1:])
    return off + np.uint64(lead), lens


def _gapped(lens, gaps, lead):
    """record i starts gaps[i] bytes after record i-1 ends (record 0: lead + gaps[0])"""
    lens = np.asarray(lens, dtype=np.uint32)
    step = np.asarray(gaps, dtype=np.uint64) + np.concatenate([[0], lens[:-1]]).astype(np.uint64)
    return np.cumsum(step) + np.uint64(lead), lens


def _device(ctx, data, off, ln, shift=0, exact=False, sorted_span=False, desc_shift=False):
    """CRCs of device-resident records; the data at `shift` bytes into its
    allocation; `exact`: the allocation ends with the last record's byte;
    `sorted_span`: LSMCK_SORTED (no device-side check of the descriptors);
    `desc_shift`: off[] 8 and len[] 4 bytes into their allocations (not
    16-byte aligned: the check's element-load path)."""
    n = len(off)
    size = int(off[-1]) + int(ln[-1]) if exact else len(data)
    d = ctx.alloc(size + shift)
    d.upload(np.ascontiguousarray(data[:size]), offset=shift)
    so, sl = (8, 4) if desc_shift else (0, 0)
    d_o, d_l, out = ctx.alloc(8 * n + so), ctx.alloc(4 * n + sl), ctx.alloc(4 * n)
    out.upload(np.full(n, 0xA5A5A5A5, dtype=np.uint32))  # unwritten outputs show
    d_o.upload(off, offset=so)
    d_l.upload(ln, offset=sl)
    ctx.crc32_device(d.ptr + shift, d_o.ptr + so, d_l.ptr + sl, n, out.ptr, sorted_span=sorted_span)
    ctx.sync()
    got = out.download(np.uint32)
    for b in (d, d_o, d_l, out):
        b.free()
    return got


@pytest.fixture
def stream_ab(ctx):
    """(stream kernel alone, walking kernel alone) on the same records: the
    first would leave the outputs unwritten if the batch were declined."""
    def run(*args, **kw):
        ctx.set_option("crc_stream", 2)
        try:
            a = _device(ctx, *args, **kw)
        finally:
            ctx.set_option("crc_stream", 1)
        ctx.set_option("crc_stream", 0)
        try:
            b = _device(ctx, *args, **kw)
        finally:
            ctx.set_option("crc_stream", 1)
        return a, b
    return run


@pytest.mark.parametrize("dist,shift", [("min", 0), ("min", 3), ("short", 1), ("mixed", 0), ("mixed", 2),
                                        ("long", 0), ("zipf", 3)])
def test_packed_vs_oracle(ctx, stream_ab, dist, shift):
    rng = np.random.default_rng(zlib.crc32(f"{dist}{shift}".encode()))
    n = 40000 if dist != "long" else 1500
    if dist == "min":  # 64-byte records: two boundaries in half the chunks
        lens = np.full(n, 64)
    elif dist == "short":
        lens = rng.integers(64, 200, n)
    elif dist == "mixed":
        lens = rng.choice([64, 65, 67, 100, 127, 128, 129, 191, 192, 255, 256, 1000, 4096, 9000], n)
    elif dist == "long":  # records over many tiles and across wave cuts
        lens = rng.integers(20000, 300000, n)
    else:
        from lsm_storage_engine_amd.device import gen_zipf_lengths
        lens = gen_zipf_lengths(77, n)
    lead = int(rng.integers(0, 300))
    off, ln = _packed(lens, lead)
    data = O.gen_stream(0x57AE0000 + shift, 0, int(off[-1]) + int(ln[-1]) + 16)
    want = O.crc32_batch(data, off, ln, threads=8)
    a, b = stream_ab(data, off, ln, shift=shift)
    assert np.array_equal(a, want)
    assert np.array_equal(b, want)


@pytest.mark.parametrize("lens,lead", [([64], 0), ([64], 77), ([1 << 20], 5), ([128] * 700, 0), ([128] * 700, 64),
                                       ([192, 64] * 500, 0), ([64] * 129 + [8192] * 3, 0), ([100] * 3, 127)])
def test_boundary_positions(ctx, stream_ab, lens, lead):
    """One record; records on the 128-byte grid (every boundary at chunk byte
    0, or at byte 64: a chain start); 64-byte records over a whole tile."""
    off, ln = _packed(lens, lead)
    data = O.gen_stream(0x57AE0100 + lead, 0, int(off[-1]) + int(ln[-1]) + 8)
    want = O.crc32_batch(data, off, ln)
    a, b = stream_ab(data, off, ln)
    assert np.array_equal(a, want) and np.array_equal(b, want)


def test_allocation_ends_with_last_record(ctx):
    """The last record ends the allocation, at every alignment: the chunk loads
    past it read zeros (buffer range), nothing beyond."""
    for end_pad in range(0, 8):
        lens = [64 + end_pad, 300, 64]
        off, ln = _packed(lens, 3)
        data = O.gen_stream(0x57AE0200 + end_pad, 0, int(off[-1]) + int(ln[-1]))
        got = _device(ctx, data, off, ln, exact=True)
        assert np.array_equal(got, O.crc32_batch(data, off, ln)), end_pad


@pytest.mark.parametrize("kind", ["wal", "gaps", "short_mixed", "empties", "tiny"])
def test_gapped_batches_vs_oracle(ctx, stream_ab, kind):
    """Records with gaps between them: WAL payloads (13- or 9-byte headers in
    between), gaps of 0..64 bytes, records under 64 bytes among long ones
    (checksummed by their window lane), empty records at their predecessor's
    end, and tiles of hundreds of tiny records (several windows per tile).
    The stream kernel alone takes every one of these batches."""
    rng = np.random.default_rng(zlib.crc32(kind.encode()))
    n = 30000
    if kind == "wal":
        lens = rng.choice([5, 17, 40, 63, 64, 65, 100, 128, 300, 1000, 5000, 9000], n)
        gaps = rng.choice([13, 9], n)
    elif kind == "gaps":
        lens = rng.choice([64, 65, 67, 100, 127, 128, 129, 191, 192, 255, 1000, 4096, 9000], n)
        gaps = rng.integers(0, 65, n)
    elif kind == "short_mixed":
        lens = np.where(rng.random(n) < 0.5, rng.integers(1, 64, n), rng.integers(64, 3000, n))
        gaps = rng.integers(0, 20, n)
    elif kind == "empties":
        lens = rng.choice([0, 0, 1, 3, 63, 64, 200, 4000], n)
        gaps = np.where(lens == 0, 0, rng.integers(0, 14, n))
        lens[0] = 77
    else:  # tiny: ~250 records per 8 KiB tile
        lens = rng.integers(1, 40, n * 4)
        gaps = rng.choice([13, 9, 0], n * 4)
    off, ln = _gapped(lens, gaps, int(rng.integers(0, 300)))
    data = O.gen_stream(0x57AE0600 + len(kind), 0, int(off[-1]) + int(ln[-1]) + 16)
    want = O.crc32_batch(data, off, ln, threads=8)
    a, b = stream_ab(data, off, ln, shift=int(rng.integers(0, 4)))
    assert np.array_equal(a, want)
    assert np.array_equal(b, want)


def test_short_records_at_page_and_allocation_edges(ctx, stream_ab):
    """Records of 1..63 bytes starting 0..15 bytes after 4 KiB boundaries of a
    page-aligned device buffer (long records with small gaps in between), and
    batches whose last record is short and ends the allocation: the window lane
    loads only the dwords that hold record bytes."""
    off, ln = [], []
    end = 0
    for page in range(1, 60):
        s = page * 4096 + page % 16          # the short record's start
        off.append(end + 5)                  # a long record up to 3 bytes before it
        ln.append(s - 3 - (end + 5))
        off.append(s)
        ln.append(1 + page % 63)
        end = s + ln[-1]
    off, ln = np.asarray(off, dtype=np.uint64), np.asarray(ln, dtype=np.uint32)
    data = O.gen_stream(0x57AE0700, 0, int(off[-1]) + int(ln[-1]) + 16)
    want = O.crc32_batch(data, off, ln)
    a, b = stream_ab(data, off, ln)
    assert np.array_equal(a, want) and np.array_equal(b, want)
    for end_pad in range(0, 8):
        off2, ln2 = _gapped([200, 63 - end_pad, 5 + end_pad], [0, 13, 9], 3)
        data2 = O.gen_stream(0x57AE0800 + end_pad, 0, int(off2[-1]) + int(ln2[-1]))
        ctx.set_option("crc_stream", 2)
        try:
            got = _device(ctx, data2, off2, ln2, exact=True)
        finally:
            ctx.set_option("crc_stream", 1)
        assert np.array_equal(got, O.crc32_batch(data2, off2, ln2)), end_pad


@pytest.mark.parametrize("case", ["overlap", "unsorted", "gap65", "empty_with_gap", "empty_first"])
def test_ineligible_batches_take_the_walking_kernel(ctx, case):
    """A caller's batch the stream kernel cannot read safely or in order --
    overlapping or unsorted records, a gap over 64 bytes, an empty record away
    from its predecessor's end, an empty first record: it declines (decided on
    the device) and the walking kernel's results are exact."""
    rng = np.random.default_rng(5)
    lens = rng.integers(64, 3000, 5000)
    off, ln = _packed(lens, 0)
    if case == "overlap":
        off[2500] -= np.uint64(1)
    elif case == "unsorted":
        off[[10, 20]] = off[[20, 10]]
        ln[[10, 20]] = ln[[20, 10]]
    elif case == "gap65":
        off[2500:] += np.uint64(65)
    elif case == "empty_with_gap":
        off[2500:] += np.uint64(3)
        ln[2500] = 0
    else:
        ln[0] = 0
    data = O.gen_stream(0x57AE0300, 0, int(off.max()) + 4000)
    got = _device(ctx, data, off, ln)
    assert np.array_equal(got, O.crc32_batch(data, off, ln, threads=8))
    ctx.set_option("crc_stream", 2)  # the stream kernel alone declines: nothing written
    try:
        assert (_device(ctx, data, off, ln) == 0xA5A5A5A5).all()
    finally:
        ctx.set_option("crc_stream", 1)


@pytest.mark.parametrize("desc_shift", [False, True])
def test_check_positions_and_descriptor_alignment(ctx, desc_shift):
    """The device check reads four records per thread (16-byte loads when the
    descriptor arrays allow them, element loads otherwise): batches of 1..4099
    records are taken, and one overlap at any position -- each slot of a
    thread's four, across threads, waves and workgroups, the last record --
    is caught."""
    rng = np.random.default_rng(23)
    for n in (1, 2, 3, 5, 4099):
        lens = rng.integers(64, 400, n)
        off, ln = _packed(lens, 5)
        data = O.gen_stream(0x57AE0A00 + n, 0, int(off[-1]) + int(ln[-1]) + 16)
        ctx.set_option("crc_stream", 2)
        try:
            got = _device(ctx, data, off, ln, desc_shift=desc_shift)
        finally:
            ctx.set_option("crc_stream", 1)
        assert np.array_equal(got, O.crc32_batch(data, off, ln)), n
    lens = rng.integers(64, 400, 4099)
    off0, ln = _packed(lens, 5)
    data = O.gen_stream(0x57AE0B00, 0, int(off0[-1]) + int(ln[-1]) + 16)
    want = O.crc32_batch(data, off0, ln, threads=8)
    for p in (1, 2, 3, 4, 5, 252, 255, 256, 257, 1023, 1024, 1025, 4098):
        off = off0.copy()
        off[p] -= np.uint64(1)  # record p overlaps record p - 1 by one byte
        want_p = want.copy()
        want_p[p] = O.crc32_batch(data, off[p:p + 1], ln[p:p + 1])[0]
        assert np.array_equal(_device(ctx, data, off, ln, desc_shift=desc_shift), want_p), p
        ctx.set_option("crc_stream", 2)  # the stream kernel alone declines: nothing written
        try:
            assert (_device(ctx, data, off, ln, desc_shift=desc_shift) == 0xA5A5A5A5).all(), p
        finally:
            ctx.set_option("crc_stream", 1)


@pytest.mark.parametrize("kind", ["packed", "wal_big_gaps"])
def test_caller_asserted_sorted_batches(ctx, kind):
    """LSMCK_SORTED: the caller asserts the order and the readable span, the
    stream kernel takes the batch without the device check -- also with gaps
    the check would refuse (a batch inside one allocation)."""
    rng = np.random.default_rng(17)
    n = 20000
    lens = rng.integers(0, 5000, n)
    lens[0] = 100
    gaps = np.zeros(n, dtype=np.int64) if kind == "packed" else rng.integers(0, 3000, n)
    off, ln = _gapped(lens, gaps, 11)
    data = O.gen_stream(0x57AE0900, 0, int(off[-1]) + int(ln[-1]) + 16)
    want = O.crc32_batch(data, off, ln, threads=8)
    ctx.set_option("crc_stream", 2)
    try:
        got = _device(ctx, data, off, ln, sorted_span=True)
    finally:
        ctx.set_option("crc_stream", 1)
    assert np.array_equal(got, want)


def test_host_batches_use_it_too(ctx):
    """Host arrays go through the staging slots in chunks; each chunk is a
    packed batch of its own (offsets rebased) and takes the stream kernel."""
    rng = np.random.default_rng(6)
    off, ln = _packed(rng.integers(64, 5000, 60000), 11)
    data = O.gen_stream(0x57AE0400, 0, int(off[-1]) + int(ln[-1]) + 8)
    assert np.array_equal(ctx.crc32(data, off, ln), O.crc32_batch(data, off, ln, threads=8))
