"""The pipelined device WAL replay ("wal_pipe": the log walked in parts on a
CU-masked stream while the previous part's CRC pass runs on the other CUs)
against the oracle's restatement of wal.rs:68-84,122-163: the same records,
status and (bad_index, bad_crc, bad_expected) triple as the unpipelined
replay, for every way the records leave (a pageable host array, a page-locked
one read back part by part on the SDMA engines, the caller's device array),
wide and compact, clean and corrupted (payload bytes, stored CRCs, type
bytes, cuts, header lengths -- a bad record at a part's last record whose
CRC span is its payload alone), and the two ways a part hands back to the
plain replay (its segment walk declines; its records outgrow the caller's
device array)."""
import numpy as np
import pytest

from lsm_storage_engine_amd.device import WAL_REC16_DTYPE, WAL_REC_DTYPE, decode_rec16
from oracle import oracle as O

from test_gpu_wal_lengths import _binary_log, length_cases

pytestmark = pytest.mark.gpu

DEFAULTS = (("wal_pipe", 0), ("wal_pipe_min", 1 << 30), ("wal_pipe_first", 4), ("wal_pipe_cus", 32),
            ("wal_pipe_layout", 0), ("wal_pipe_seg", 0), ("wal_seg_bytes", 0), ("wal_seg_rounds", 16),
            ("wal_seg_prepair", 2), ("wal_seg_pack", 1), ("wal_dma_engines", 4))


@pytest.fixture
def opts(ctx):
    def set_(**kw):
        for k, v in kw.items():
            ctx.set_option(k, v)
    yield set_
    for k, v in DEFAULTS:
        ctx.set_option(k, v)


def rows(recs, compact):
    if compact:
        f = decode_rec16(recs)
        return list(zip(*(np.asarray(f[k]).tolist() for k in ("rec_off", "payload_off", "klen", "vlen", "type"))))
    return list(zip(*(np.asarray(recs[k]).tolist() for k in ("rec_off", "payload_off", "klen", "vlen", "type",
                                                              "crc"))))


def oracle_rows(orecs, compact):
    if compact:
        return [(r.rec_off, r.payload_off, r.klen, r.vlen, r.type) for r in orecs]
    return [(r.rec_off, r.payload_off, r.klen, r.vlen, r.type, r.crc) for r in orecs]


def replay(ctx, d, img, mode, compact, cap=None):
    """(status, rows, bad) of the device image in d: records to a pageable or
    pinned host array, or to a device array (mode 'dev')."""
    n = len(img)
    if mode == "dev":
        RD = WAL_REC16_DTYPE if compact else WAL_REC_DTYPE
        cap = cap or n // 9 + 1
        out = ctx.alloc(cap * RD.itemsize)
        try:
            m, st, bad = ctx.wal_replay_verify_to_device(n, out.ptr, cap, device_ptr=d.ptr, compact=compact)
            got = out.download(np.uint8, cap * RD.itemsize).view(RD)[:min(m, cap)]
        finally:
            out.free()
        return st, rows(got, compact), bad
    recs, st, bad = ctx.wal_replay_verify(n, device_ptr=d.ptr, cap=cap, pinned_recs=mode == "pinned", compact=compact)
    r = rows(recs.copy(), compact)
    del recs
    return st, r, bad


def check(ctx, img, mode, compact, cap=None, name=""):
    d = ctx.alloc(max(1, len(img)))
    try:
        d.upload(np.frombuffer(img, np.uint8))
        st, got, bad = replay(ctx, d, img, mode, compact, cap)
    finally:
        d.free()
    ost, orecs, obad = O.wal_replay(img)
    assert st == ost, name
    want = oracle_rows(orecs, compact)
    assert got == (want if cap is None else want[:cap]), name
    if st:
        k = 2 if st == 3 else 3
        assert tuple(bad[:k]) == tuple(obad[:k]), name
    return st


@pytest.fixture(scope="module")
def log():
    img = _binary_log(15000, 2024)
    return img, length_cases(img)


def _part_end_cases(ctx, img, opts_set):
    """Corruptions at the records that end the pipeline's parts (their CRC
    spans are their payloads alone): the stored CRC flipped, the payload
    flipped.  The part ends follow from the walk; each bound lim gives the
    last record that starts before it."""
    st, R, _ = O.wal_replay(img)
    n = len(img)
    first, parts = opts_set["wal_pipe_first"], opts_set["wal_pipe"]
    a0 = max(n * first // 64, 1)
    lims = [a0] + [a0 + (n - a0) * k // (parts - 1) for k in range(1, parts - 1)]
    starts = [r.rec_off for r in R]
    out = []
    for lim in lims:
        i = int(np.searchsorted(starts, lim, side="left")) - 1  # the last record starting before lim
        if i < 0 or R[i].klen + R[i].vlen == 0:
            continue
        b = bytearray(img)
        b[R[i].rec_off + 1] ^= 0x04
        out.append(("part end stored crc", bytes(b)))
        b = bytearray(img)
        b[R[i].payload_off] ^= 0x80
        out.append(("part end payload", bytes(b)))
    return out


@pytest.mark.parametrize("compact", [True, False])
@pytest.mark.parametrize("mode", ["pageable", "pinned", "dev"])
@pytest.mark.parametrize("parts,first,layout", [(2, 8, 0), (5, 1, 1), (16, 4, 0)])
def test_pipe_equals_oracle(ctx, opts, log, mode, compact, parts, first, layout):
    o = {"wal_pipe": parts, "wal_pipe_min": 1 << 20, "wal_pipe_first": first, "wal_pipe_layout": layout}
    opts(**o)
    img, cases = log
    assert check(ctx, img, mode, compact, name="clean") == 0
    assert ctx.get_stat("wal_pipe_parts") == parts
    assert ctx.get_stat("wal_walk_path") == 1
    if mode == "pinned":
        assert 1 <= ctx.get_stat("wal_recs_dma") <= 4
    for name, im in _part_end_cases(ctx, img, o):
        check(ctx, im, mode, compact, name=name)
    for name, im in cases[::3] if mode != "pinned" else cases:
        check(ctx, im, mode, compact, name=name)


@pytest.mark.parametrize("cus,seg", [(8, 0), (64, 0), (32, 4096)])
def test_pipe_walk_cus_and_segments(ctx, opts, log, cus, seg):
    """The walk on 8 or 64 CUs, parts in forced 4 KiB segments."""
    opts(wal_pipe=6, wal_pipe_min=1 << 20, wal_pipe_cus=cus, wal_pipe_seg=seg)
    img, cases = log
    assert check(ctx, img, "pinned", True) == 0
    assert ctx.get_stat("wal_pipe_parts") == 6
    for name, im in cases[1::4]:
        check(ctx, im, "pinned", True, name=name)


def test_pipe_cap_below_count(ctx, opts, log):
    """cap below the record count: host arrays get cap records (the parts past
    cap read back nothing); a device array that the parts outgrow hands the
    replay back to the plain path (wal_pipe_parts 0) with the same result."""
    opts(wal_pipe=4, wal_pipe_min=1 << 20)
    img, _ = log
    for mode in ("pageable", "pinned"):
        assert check(ctx, img, mode, True, cap=7000) == 0
        assert ctx.get_stat("wal_pipe_parts") == 4
    assert check(ctx, img, "dev", True, cap=7000) == 0
    assert ctx.get_stat("wal_pipe_parts") == 0


def test_pipe_decline_to_plain(ctx, opts):
    """A log of logs in 256-byte segments with no repair rounds: a part's
    segment walk declines, the replay starts over unpipelined (candidate
    doubling) -- the oracle's records either way."""
    inner = _binary_log(60, 63)[:6000]
    rng = np.random.default_rng(64)
    img = b"".join(O.wal_insert(b"k%d" % i, inner if i % 3 == 0 else rng.bytes(int(rng.integers(0, 400))))
                   for i in range(3000))
    opts(wal_pipe=4, wal_pipe_min=1 << 16, wal_seg_bytes=256, wal_seg_rounds=0, wal_seg_prepair=0)
    assert check(ctx, img, "pinned", True) == 0
    # (a declined part: the plain replay, whose own segment walk declines too)
    assert (ctx.get_stat("wal_pipe_parts") == 0) == (ctx.get_stat("wal_walk_path") == 2)


def test_pipe_packed_off(ctx, opts, log):
    """Payload-only CRC spans (wal_seg_pack 0) through the pipeline."""
    opts(wal_pipe=3, wal_pipe_min=1 << 20, wal_seg_pack=0)
    img, cases = log
    assert check(ctx, img, "pinned", False) == 0
    for name, im in cases[::5]:
        check(ctx, im, "pinned", False, name=name)


def test_pipe_hipmemcpy_readback(ctx, opts, log):
    """wal_dma_engines 0: no part-by-part read-back; wal_finish reads every
    record back after the last part."""
    opts(wal_pipe=4, wal_pipe_min=1 << 20, wal_dma_engines=0)
    img, cases = log
    for mode in ("pinned", "pageable"):
        assert check(ctx, img, mode, True) == 0
        assert ctx.get_stat("wal_recs_dma") == 0
    check(ctx, cases[0][1], "pinned", True)


def test_pipe_1gib(ctx, opts):
    """A 1 GiB log of 100-8000 B records in 8 parts, records to a pinned host
    array and to HBM, clean and with a bad record in the fifth part."""
    from test_gpu_wal_lengths import _big_log
    img = _big_log(1 << 30, 78)
    opts(wal_pipe=8)
    st, R, _ = O.wal_replay(img)
    assert st == 0
    for mode in ("pinned", "dev"):
        assert check(ctx, img, mode, True, cap=len(R) + 8) == 0
        assert ctx.get_stat("wal_pipe_parts") == 8
    b = bytearray(img)
    r = next(r for r in R[len(R) * 5 // 8:] if r.type == 1 and r.vlen)
    b[r.payload_off + r.klen] ^= 0x02
    assert check(ctx, bytes(b), "pinned", True, cap=len(R) + 8) == 1
