"""Corrupted header LENGTHS through every GPU WAL walk, against the oracle's
restatement of wal.rs:122-163.

A record's klen / vlen decide where the next header is (wal.rs:127-132:
``data_len = key_len + val_len`` in u32, then ``take(data_len)``), so a
damaged length moves the whole chain after it: the riskiest input for a
speculative parallel header walk.  Each case below is replayed by the segment
walk (auto and forced segment sizes, no repair rounds), candidate doubling,
the walk in parts, the host walk of a device image, the host walk of a host
image, the GPU walk of an uploaded host image and the split upload -- wide
(lsmck_wal_rec) and compact (lsmck_wal_rec16) records -- and must give the
oracle's status, records and (bad_index, bad_crc, bad_expected) triple:

  (a) bit flips in klen / vlen of mid-log Insert and Remove records, low bits
      (the chain moves a little) and high bits (the length runs past EOF:
      take() returns the short rest, wal.rs:132);
  (b) a length rewritten so the next "header" is a payload byte equal to a
      valid command type;
  (c) the u32 wrap of klen + vlen (wal.rs:129: 0xFFFFFFF0 + 0x20 = 0x10);
  (d) a length that skips exactly one record;
and, for each, the stored CRC either kept (the record itself fails) or refit
to the bytes the new length covers (the record passes and the walk goes on
from where the damaged length points -- the reference's chain, not the
original one).  One ≥ 1 GiB log repeats (a), (c) and (d) at full scale.
"""
import zlib

import numpy as np
import pytest

from lsm_storage_engine_amd.device import decode_rec16
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEFAULTS = (("wal_seg_bytes", 0), ("wal_seg_rounds", 16), ("wal_seg_walk", 1), ("wal_seg_pack", 1),
            ("wal_seg_stage", 1), ("wal_seg_prepair", 2), ("wal_part_bytes", 0), ("wal_gpu_walk", 1),
            ("wal_upload_min", 1 << 20), ("wal_split", 1), ("wal_stage_bytes", 16 << 20))

# name -> (image where, options)
PATHS = {
    "seg_auto": ("device", {}),
    "seg_64": ("device", {"wal_seg_bytes": 64}),
    "seg_512": ("device", {"wal_seg_bytes": 512}),
    "seg_4k": ("device", {"wal_seg_bytes": 4096}),
    "seg_256k": ("device", {"wal_seg_bytes": 262144}),
    "seg_norepair": ("device", {"wal_seg_bytes": 512, "wal_seg_rounds": 0, "wal_seg_prepair": 0}),
    "seg_nostage": ("device", {"wal_seg_stage": 0, "wal_seg_pack": 0}),
    "doubling": ("device", {"wal_seg_walk": 0}),
    "parts_1m": ("device", {"wal_part_bytes": 1 << 20}),
    "device_hostwalk": ("device", {"wal_gpu_walk": 0}),
    "host_walk": ("host", {"wal_upload_min": 0}),
    "host_upload": ("host", {"wal_upload_min": 1}),
    "host_split": ("host", {"wal_upload_min": 1, "wal_stage_bytes": 1 << 20, "wal_split": 1}),
}


@pytest.fixture
def opts(ctx):
    def set_(**kw):
        for k, v in kw.items():
            ctx.set_option(k, v)
    yield set_
    for k, v in DEFAULTS:
        ctx.set_option(k, v)


def _u32(b, at):
    return int.from_bytes(bytes(b[at:at + 4]), "little")


def _put(b, at, v):
    b[at:at + 4] = (v & 0xFFFFFFFF).to_bytes(4, "little")


def _refit(b, rec_off):
    """Rewrites the stored CRC of the record at rec_off to the CRC of the
    bytes its (damaged) header lengths now cover, as next_record reads them
    (wal.rs:127-135: u32 data_len, take() short at EOF)."""
    t = b[rec_off]
    hdr = 13 if t == 1 else 9
    dlen = (_u32(b, rec_off + 5) + (_u32(b, rec_off + 9) if t == 1 else 0)) & 0xFFFFFFFF
    p = rec_off + hdr
    _put(b, rec_off + 1, zlib.crc32(bytes(b[p:p + dlen])))


def _binary_log(n, seed):
    """Insert / Remove records with random binary keys and values (bytes 1 and
    2 everywhere: bogus header candidates for the walks), ~5 MiB."""
    rng = np.random.default_rng(seed)
    blob = rng.bytes(1 << 21)
    parts = []
    for i in range(n):
        kl, vl = int(rng.integers(2, 40)), int(rng.integers(24, 640))
        o = int(rng.integers(0, (1 << 21) - 700))
        k = blob[o:o + kl]
        parts.append(O.wal_remove(k) if i % 9 == 0 else O.wal_insert(k, blob[o + 40:o + 40 + vl]))
    return b"".join(parts)


def _wrap_record(klen, vlen, payload, fit=True):
    """An Insert whose u32 klen + vlen wraps to len(payload) (wal.rs:129)."""
    assert (klen + vlen) & 0xFFFFFFFF == len(payload)
    crc = zlib.crc32(payload) if fit else zlib.crc32(payload) ^ 0x5A5A5A5A
    return bytes([1]) + crc.to_bytes(4, "little") + klen.to_bytes(4, "little") + vlen.to_bytes(4, "little") + payload


def length_cases(img):
    """[(name, image)]: the header-length corruptions (a)-(d) of a clean log."""
    st, R, _ = O.wal_replay(img)
    assert st == 0
    n = len(R)
    mid = range(n // 3, n - 4)
    ins = [i for i in mid if R[i].type == 1 and R[i].klen >= 2 and R[i].vlen >= 24 and R[i + 1].type == 1]
    rem = [i for i in mid if R[i].type == 2 and R[i].klen >= 2]
    end = lambda i: R[i + 1].rec_off if i + 1 < n else len(img)  # noqa: E731
    out = []

    def edit(name, i, field, fn, refit):
        b = bytearray(img)
        at = R[i].rec_off + (5 if field == "klen" else 9)
        _put(b, at, fn(_u32(b, at)))
        if refit:
            _refit(b, R[i].rec_off)
        out.append((name + ("/refit" if refit else "/kept"), bytes(b)))

    for refit in (False, True):
        # (a) bit flips: low bits move the chain a little, high bits run it past EOF
        edit("a_ins_klen_bit0", ins[3], "klen", lambda v: v ^ 0x1, refit)
        edit("a_ins_vlen_bit4", ins[40], "vlen", lambda v: v ^ 0x10, refit)
        edit("a_ins_vlen_bit16", ins[77], "vlen", lambda v: v ^ 0x10000, refit)
        edit("a_ins_vlen_bit31", ins[len(ins) // 2], "vlen", lambda v: v ^ 0x80000000, refit)
        edit("a_ins_klen_bit24", ins[len(ins) // 3], "klen", lambda v: v ^ 0x01000000, refit)
        edit("a_rem_klen_bit1", rem[5], "klen", lambda v: v ^ 0x2, refit)
        edit("a_rem_klen_bit31", rem[len(rem) // 2], "klen", lambda v: v ^ 0x80000000, refit)
        # (d) a length that skips exactly one record (the record after it hidden in its payload)
        i = ins[100]
        edit("d_ins_skip_one", i, "vlen", lambda v, i=i: v + end(i + 1) - R[i + 1].rec_off, refit)
        j = rem[20]
        edit("d_rem_skip_one", j, "klen", lambda v, j=j: v + end(j + 1) - R[j + 1].rec_off, refit)
        # first and last records
        edit("a_first_klen", 0, "klen", lambda v: v ^ 0x4, refit)
        last = n - 1 if R[n - 1].type == 1 else n - 2
        edit("a_last_vlen_past_eof", last, "vlen", lambda v: v + 5, refit)
        # zero lengths: the next header is read at the payload's first byte
        edit("a_ins_zero", ins[200], "klen", lambda v: 0, refit)
        if not refit:
            continue
        b = bytearray(img)
        _put(b, R[ins[200]].rec_off + 9, 0)
        _refit(b, R[ins[200]].rec_off)
        out.append(("a_ins_both_zero/refit", bytes(b)))

    # (b) the next "header" lands on a payload byte that is a valid type: in
    # the following record's payload (length grown) or in its own (shrunk)
    for grow in (True, False):
        for i in ins[300:]:
            p = R[i].payload_off
            lo, hi = (R[i + 1].payload_off + 1, end(i + 1)) if grow else (p + R[i].klen + 1, end(i))
            q = next((q for q in range(lo, hi) if img[q] in (1, 2)), None)
            if q is None:
                continue
            for refit in (False, True):
                b = bytearray(img)
                _put(b, R[i].rec_off + 9, q - p - R[i].klen)
                if refit:
                    _refit(b, R[i].rec_off)
                out.append((f"b_lands_on_type_{'grow' if grow else 'shrink'}/{'refit' if refit else 'kept'}",
                            bytes(b)))
            break

    # (c) the u32 wrap of klen + vlen, a record put in front of a mid-log record
    at = R[n // 2].rec_off
    pay16, pay8 = bytes(range(16)), b"wrapwrap"
    for name, rec in (("c_wrap_klen_big/refit", _wrap_record(0xFFFFFFF0, 0x20, pay16)),
                      ("c_wrap_klen_big/kept", _wrap_record(0xFFFFFFF0, 0x20, pay16, fit=False)),
                      ("c_wrap_vlen_big/refit", _wrap_record(0x10, 0xFFFFFFF8, pay8)),
                      ("c_wrap_klen_max/refit", _wrap_record(0xFFFFFFFF, 0xF, bytes(pay16[:14])))):
        out.append((name, img[:at] + rec + img[at:]))
    # a record whose lengths wrap, rewritten in place (the chain goes on inside its old payload)
    i = ins[400]
    for refit in (False, True):
        b = bytearray(img)
        _put(b, R[i].rec_off + 5, 0xFFFFFFF0)
        _put(b, R[i].rec_off + 9, 0x18)
        if refit:
            _refit(b, R[i].rec_off)
        out.append(("c_wrap_in_place/" + ("refit" if refit else "kept"), bytes(b)))
    return out


def replay(ctx, img, where, compact, shift=0):
    """(status, records as tuples, bad triple) from the GPU library."""
    if where == "device":
        d = ctx.alloc(max(1, len(img)) + shift)
        try:
            if img:
                d.upload(np.frombuffer(img, np.uint8), offset=shift)
            recs, st, bad = ctx.wal_replay_verify(len(img), device_ptr=d.ptr + shift, compact=compact)
            recs = recs.copy()
        finally:
            d.free()
    else:
        recs, st, bad = ctx.wal_replay_verify(img, compact=compact)
        recs = recs.copy()
    if compact:
        f = decode_rec16(recs)
        rows = list(zip(*(np.asarray(f[k]).tolist() for k in ("rec_off", "payload_off", "klen", "vlen", "type"))))
    else:
        rows = list(zip(*(np.asarray(recs[k]).tolist() for k in ("rec_off", "payload_off", "klen", "vlen", "type",
                                                                  "crc"))))
    return st, rows, bad


def oracle_rows(orecs, compact):
    if compact:
        return [(r.rec_off, r.payload_off, r.klen, r.vlen, r.type) for r in orecs]
    return [(r.rec_off, r.payload_off, r.klen, r.vlen, r.type, r.crc) for r in orecs]


def check(ctx, name, img, where, compact, shift=0):
    st, rows, bad = replay(ctx, img, where, compact, shift)
    ost, orecs, obad = O.wal_replay(img)
    assert st == ost, name
    assert rows == oracle_rows(orecs, compact), name
    if st:
        k = 2 if st == 3 else 3  # InvalidCommandType reports the index and the byte
        assert tuple(bad[:k]) == tuple(obad[:k]), name
    return st


@pytest.fixture(scope="module")
def log_and_cases():
    img = _binary_log(15000, 2024)
    assert len(img) > (4 << 20)
    return img, length_cases(img)


def test_cases_cover_every_outcome(log_and_cases):
    """The cases reach every outcome of next_record: a clean end (status 0),
    CorruptedData (1), the Remove panic (2) and InvalidCommandType (3)."""
    _, cases = log_and_cases
    seen = {O.wal_replay(im)[0] for _, im in cases}
    assert seen == {0, 1, 2, 3}, seen
    assert len(cases) >= 30


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("path", list(PATHS))
def test_corrupted_lengths(ctx, opts, log_and_cases, path, compact):
    where, o = PATHS[path]
    opts(**o)
    img, cases = log_and_cases
    assert check(ctx, "clean", img, where, compact) == 0
    if path.startswith("seg_"):  # the walk the path names ran
        assert ctx.get_stat("wal_walk_path") in ((1, 2) if path == "seg_norepair" else (1,))
    elif path in ("doubling", "parts_1m"):  # (a part size: candidate doubling in parts)
        assert ctx.get_stat("wal_walk_path") == 2
    for name, im in cases:
        check(ctx, name, im, where, compact)


@pytest.mark.parametrize("path", ["seg_auto", "seg_64", "doubling"])
def test_corrupted_lengths_unaligned(ctx, opts, log_and_cases, path):
    """The same cases with the device image at an odd address."""
    where, o = PATHS[path]
    opts(**o)
    img, cases = log_and_cases
    for name, im in cases:
        check(ctx, name, im, where, compact=True, shift=3)


def _big_log(target, seed):
    """A ≥ target-byte WAL image of Insert / Remove records of 100-8000 B of
    random bytes."""
    rng = np.random.default_rng(seed)
    blob = rng.bytes(16 << 20)
    parts, total, i = [], 0, 0
    while total < target:
        vl = int(rng.integers(100, 8000))
        o = int(rng.integers(0, (16 << 20) - vl - 32))
        r = O.wal_remove(blob[o:o + 24]) if i % 11 == 0 else O.wal_insert(blob[o:o + 16], blob[o + 16:o + 16 + vl])
        parts.append(r)
        total += len(r)
        i += 1
    return b"".join(parts)


def test_corrupted_length_1gib(ctx, opts):
    """One corrupted length in a ≥ 1 GiB log (device image, compact records;
    the host image through the split upload for one case): a length that skips
    one record (refit), a high bit flipped in a vlen (the CRC runs over the
    rest of the log and fails), the same refit (the record swallows the rest of
    the log), and a record whose lengths wrap in u32 -- the oracle's outcome."""
    img = _big_log(1 << 30, 77)
    st, R, _ = O.wal_replay(img)
    assert st == 0
    n = len(R)
    i = next(k for k in range(n // 2, n) if R[k].type == 1 and R[k + 1].type == 1)
    cases = []
    b = bytearray(img)
    _put(b, R[i].rec_off + 9, R[i].vlen + R[i + 2].rec_off - R[i + 1].rec_off)
    _refit(b, R[i].rec_off)
    cases.append(("skip_one/refit", bytes(b)))
    b = bytearray(img)
    _put(b, R[i].rec_off + 9, R[i].vlen ^ 0x80000000)
    cases.append(("vlen_bit31/kept", bytes(b)))
    _refit(b, R[i].rec_off)
    cases.append(("vlen_bit31/refit", bytes(b)))
    del b
    at = R[n // 3].rec_off
    cases.append(("wrap/refit", img[:at] + _wrap_record(0xFFFFFFF0, 0x20, bytes(range(16))) + img[at:]))
    want = {"skip_one/refit": 0, "vlen_bit31/kept": 1, "vlen_bit31/refit": 0, "wrap/refit": 0}
    for name, im in cases:
        assert check(ctx, name, im, "device", compact=True) == want[name]
    opts(wal_upload_min=1)
    name, im = cases[0]
    assert check(ctx, name, im, "host", compact=True) == 0
