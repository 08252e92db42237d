"""The stream kernel (crc32_stream_kernel, lsmck_crc32.hip): packed batches of
records of at least 64 bytes checksummed from aligned 128-byte chunks of the
byte stream, record boundaries as CRC register resets.  Every case is checked
against the oracle (crc 1.x's algorithm, oracle/lsmck_oracle.c) and against the
walking kernel on the same records (crc_stream 0).  tools/stream_sim.py is the
CPU model of the same algebra."""
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


def _device(ctx, data, off, ln, shift=0, exact=False):
    """CRCs of device-resident records; the data at `shift` bytes into its
    allocation; `exact`: the allocation ends with the last record's byte."""
    n = len(off)
    size = int(off[-1]) + int(ln[-1]) if exact else len(data)
    d = ctx.alloc(size + shift)
    d.upload(np.ascontiguousarray(data[:size]), offset=shift)
    d_o, d_l, out = ctx.alloc(8 * n), ctx.alloc(4 * n), ctx.alloc(4 * n)
    out.upload(np.full(n, 0xA5A5A5A5, dtype=np.uint32))  # unwritten outputs show
    d_o.upload(off)
    d_l.upload(ln)
    ctx.crc32_device(d.ptr + shift, d_o.ptr, d_l.ptr, n, out.ptr)
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
def test_packed_vs_oracle(ctx, stream_ab, sel, dist, shift):
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


@pytest.fixture(params=[(0, 0, 0, 0), (1, 0, 0, 0), (2, 0, 0, 0), (1, 1, 0, 0), (1, 1, 1, 0), (1, 1, 1, 1)],
                ids=["branch_steps", "select_steps", "branch_free", "dpp_map", "default", "spread_finish"])
def sel(ctx, request):
    """The stream kernel's boundary words: steps inside the branch (0), the
    branch selecting the step inputs (1, the default), or no branch (2); with
    and without the short path for tiles without a boundary (default: with)."""
    ctx.set_option("crc_stream_sel", request.param[0])
    ctx.set_option("crc_stream_z0", request.param[1])
    ctx.set_option("crc_stream_lm", request.param[2])
    ctx.set_option("crc_stream_fsp", request.param[3])
    yield request.param
    ctx.set_option("crc_stream_sel", 1)
    ctx.set_option("crc_stream_z0", 1)
    ctx.set_option("crc_stream_lm", 1)
    ctx.set_option("crc_stream_fsp", 0)


@pytest.mark.parametrize("lens,lead", [([64], 0), ([64], 77), ([1 << 20], 5), ([128] * 700, 0), ([128] * 700, 64),
                                       ([192, 64] * 500, 0), ([64] * 129 + [8192] * 3, 0), ([100] * 3, 127)])
def test_boundary_positions(ctx, stream_ab, sel, lens, lead):
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


@pytest.mark.parametrize("case", ["short_record", "gap", "overlap", "unsorted"])
def test_ineligible_batches_take_the_walking_kernel(ctx, case):
    """Not a packed batch of >= 64-byte records: the stream kernel declines
    (decided on the device) and the walking kernel's results are exact."""
    rng = np.random.default_rng(5)
    lens = rng.integers(64, 3000, 5000)
    off, ln = _packed(lens, 0)
    if case == "short_record":
        ln[2500] = 63
    elif case == "gap":
        off[2500:] += np.uint64(1)
    elif case == "overlap":
        off[2500] -= np.uint64(1)
    else:
        off[[10, 20]] = off[[20, 10]]
        ln[[10, 20]] = ln[[20, 10]]
    data = O.gen_stream(0x57AE0300, 0, int(off.max()) + 4000)
    got = _device(ctx, data, off, ln)
    assert np.array_equal(got, O.crc32_batch(data, off, ln, threads=8))
    ctx.set_option("crc_stream", 2)  # the stream kernel alone declines: nothing written
    try:
        assert (_device(ctx, data, off, ln) == 0xA5A5A5A5).all()
    finally:
        ctx.set_option("crc_stream", 1)


def test_host_batches_use_it_too(ctx):
    """Host arrays go through the staging slots in chunks; each chunk is a
    packed batch of its own (offsets rebased) and takes the stream kernel."""
    rng = np.random.default_rng(6)
    off, ln = _packed(rng.integers(64, 5000, 60000), 11)
    data = O.gen_stream(0x57AE0400, 0, int(off[-1]) + int(ln[-1]) + 8)
    assert np.array_equal(ctx.crc32(data, off, ln), O.crc32_batch(data, off, ln, threads=8))


@pytest.mark.parametrize("waves,ring,batch,qstore,window", [(12, 0, 0, 1, 2), (12, 3, 0, 1, 2), (0, 0, 1, 1, 2),
                                                           (12, 0, 1, 1, 2), (0, 0, 0, 0, 2), (0, 0, 0, 1, 1),
                                                           (0, 0, 0, 1, 0), (0, 0, 0, 2, 2), (0, 0, 0, 1, 2)])
def test_workgroup_and_slot_variants(ctx, waves, ring, batch, qstore, window):
    """The 12-wave workgroup form (168 VGPRs) with two and three payload slots
    in flight, the records finished in batches of 64, per-tile stores instead
    of queued 256-B blocks, and the reloaded boundary windows: same CRCs as the
    oracle."""
    rng = np.random.default_rng(8)
    lens = rng.choice([64, 65, 100, 127, 128, 129, 300, 1000, 4096, 20000], 50000)
    off, ln = _packed(lens, 13)
    data = O.gen_stream(0x57AE0500, 0, int(off[-1]) + int(ln[-1]) + 8)
    want = O.crc32_batch(data, off, ln, threads=8)
    ctx.set_option("crc_wg_waves", waves)
    ctx.set_option("crc_ring", ring)
    ctx.set_option("crc_stream_batch", batch)
    ctx.set_option("crc_stream_qstore", qstore)
    ctx.set_option("crc_stream_window", window)
    ctx.set_option("crc_stream", 2)
    try:
        got = _device(ctx, data, off, ln)
    finally:
        ctx.set_option("crc_wg_waves", 0)
        ctx.set_option("crc_ring", 0)
        ctx.set_option("crc_stream_batch", 0)
        ctx.set_option("crc_stream_qstore", 2)
        ctx.set_option("crc_stream_window", 2)
        ctx.set_option("crc_stream", 1)
    assert np.array_equal(got, want)
