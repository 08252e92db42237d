"""The segment walk (lsmck_segwalk.h, the GPU WAL header walk's logic) run on
the host through tools/segwalk_sim.cpp -- the kernels' own per-thread
functions in the launch order of lsmck_api.cpp -- against a plain chain walk
of wal.rs:68-84,122-163 (each record at the previous one's end, the payload
cut at EOF, the chain ending at EOF, in a truncated header, or at a byte that
is not a command type).  Covers what the GPU suite can afford little of:
segments far smaller than records, every cut position, bad type bytes, and
payloads built to fool the guesses (framed records inside values, floods of
type bytes), where the check must catch every wrong guess and the repairs (or
the decline to candidate doubling) must leave the chain exact."""
import ctypes as C
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lsm_storage_engine_amd", "csrc")
END, BAD = 2, 3


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("segwalk") / "libsegwalk_sim.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I", CSRC, "-o", so,
                    os.path.join(ROOT, "tools", "segwalk_sim.cpp")], check=True)
    lib = C.CDLL(so)
    u64p = C.POINTER(C.c_uint64)
    lib.segwalk_sim.restype = C.c_int
    lib.segwalk_sim.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, u64p, C.c_size_t, u64p,
                                C.POINTER(C.c_uint32), u64p, C.POINTER(C.c_int), u64p, C.POINTER(C.c_uint32)]

    def run(img, S, start=0, rounds=16, shift=0):
        raw = np.zeros(len(img) + shift + 1, dtype=np.uint8)  # shift: the image at an odd address
        a = raw[shift:shift + len(img)]
        a[:] = np.frombuffer(bytes(img), np.uint8)
        cap = len(img) // 9 + 2
        offs = (C.c_uint64 * cap)()
        m, code, pos, rep, K, nf = C.c_uint64(), C.c_uint32(), C.c_uint64(), C.c_int(), C.c_uint64(), C.c_uint32()
        rc = lib.segwalk_sim(a.ctypes.data, len(img), start, S, rounds, offs, cap, C.byref(m), C.byref(code),
                             C.byref(pos), C.byref(rep), C.byref(K), C.byref(nf))
        assert rc in (0, 1), rc
        if rc == 1:
            return None
        return list(offs[:m.value]), code.value, (pos.value if code.value == BAD else 0), rep.value
    lib.segwalk_sim_prefix.restype = C.c_int
    lib.segwalk_sim_prefix.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, u64p,
                                       C.c_size_t, u64p, C.POINTER(C.c_uint32), u64p, C.POINTER(C.c_int), u64p,
                                       C.POINTER(C.c_uint32)]

    def prefix(img, start, lim, S, rounds=16):
        """(records starting in [start, lim), code, pos): pos is where the
        next prefix starts when code is EXIT (1), the bad byte for BAD"""
        a = np.frombuffer(bytes(img), np.uint8)
        cap = len(img) // 9 + 2
        offs = (C.c_uint64 * cap)()
        m, code, pos, rep, K, nf = C.c_uint64(), C.c_uint32(), C.c_uint64(), C.c_int(), C.c_uint64(), C.c_uint32()
        rc = lib.segwalk_sim_prefix(a.ctypes.data, len(img), start, lim, S, rounds, offs, cap, C.byref(m),
                                    C.byref(code), C.byref(pos), C.byref(rep), C.byref(K), C.byref(nf))
        assert rc in (0, 1), rc
        return None if rc == 1 else (list(offs[:m.value]), code.value, pos.value)
    run.prefix = prefix
    lib.segwalk_sim_set_nsub.argtypes = [C.c_uint32]
    run.set_nsub = lib.segwalk_sim_set_nsub
    lib.segwalk_sim_set_stage.argtypes = [C.c_uint32]
    run.set_stage = lib.segwalk_sim_set_stage
    lib.segwalk_sim_pack.argtypes = [u64p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_size_t]
    lib.segwalk_sim_unpack.restype = C.c_uint32
    lib.segwalk_sim_unpack.argtypes = [C.c_uint32] * 5

    def packed(img, S):
        """the walk's packed CRC spans (seg::Pack): (offs, lens, expected CRCs)"""
        cap = len(img) // 9 + 2
        po, pl, pe = (C.c_uint64 * cap)(), (C.c_uint32 * cap)(), (C.c_uint32 * cap)()
        lib.segwalk_sim_pack(po, pl, pe, cap)
        try:
            res = run(img, S)
        finally:
            lib.segwalk_sim_pack(None, None, None, 0)
        m = len(res[0])
        return list(po[:m]), list(pl[:m]), list(pe[:m])
    run.unpack = lib.segwalk_sim_unpack
    run.packed = packed
    lib.segwalk_sim_set_prepair.argtypes = [C.c_int]
    run.set_prepair = lib.segwalk_sim_set_prepair
    lib.segwalk_sim_prepairs.restype = C.c_int
    run.prepairs = lib.segwalk_sim_prepairs
    return run


def chain(img, start=0):
    """wal.rs's read loop over the headers alone (no CRCs)."""
    n, p, offs = len(img), start, []
    while True:
        if p >= n:
            return offs, END, 0
        t = img[p]
        if t not in (1, 2):
            return offs, BAD, p
        h = 13 if t == 1 else 9
        if p + h > n:
            return offs, END, 0
        klen = struct.unpack_from("<I", img, p + 5)[0]
        vlen = struct.unpack_from("<I", img, p + 9)[0] if t == 1 else 0
        dlen = (klen + vlen) & 0xFFFFFFFF
        offs.append(p)
        p += h + min(dlen, n - p - h)


def rec(key, val=None):
    if val is None:
        return struct.pack("<BII", 2, 0x1234, len(key)) + key
    return struct.pack("<BIII", 1, 0x5678, len(key), len(val)) + key + val


def random_log(rng, nrec, lo=0, hi=600, remove_every=9):
    parts = []
    for i in range(nrec):
        kl = int(rng.integers(0, 40))
        vl = int(rng.integers(lo, hi))
        k = rng.bytes(kl)
        parts.append(rec(k) if i % remove_every == 0 else rec(k, rng.bytes(vl)))
    return bytearray(b"".join(parts))


def check(sim, img, S, start=0, shift=0, rounds=16, expect_fast=True):
    want = chain(bytes(img), start)
    got = sim(img, S, start=start, rounds=rounds, shift=shift)
    if got is None:
        assert not expect_fast, "declined"
        return None
    offs, code, pos, rep = got
    assert code == want[1] and pos == want[2]
    assert offs == want[0]
    return rep


@pytest.mark.parametrize("S", [64, 100, 512, 4096, 1 << 16, 1 << 17, 1 << 19])
@pytest.mark.parametrize("shift", [0, 3])
def test_random_logs(sim, S, shift):
    rng = np.random.default_rng(S + shift)
    img = random_log(rng, 3000)
    rep = check(sim, img, S, shift=shift)
    if S >= 1024:  # every segment holds a true record start: no wrong guess to repair
        assert rep == 0


def test_long_records_span_segments(sim):
    rng = np.random.default_rng(7)
    parts = [rec(rng.bytes(8), rng.bytes(int(L))) for L in rng.integers(0, 20000, 300)]
    img = bytearray(b"".join(parts))
    for S in (64, 1000, 4096):
        assert check(sim, img, S) is not None


def test_every_cut_position(sim):
    """Truncated logs: EOF inside a header (clean end) or inside a payload
    (the record kept with a short payload) -- the true entry of the last
    segment may be refused by the guess, and the check repairs it."""
    rng = np.random.default_rng(11)
    img = random_log(rng, 40, hi=200)
    for cut in range(0, len(img) + 1):
        check(sim, img[:cut], 128)


def test_bad_type_bytes(sim):
    rng = np.random.default_rng(12)
    img = random_log(rng, 2000)
    offs = chain(bytes(img))[0]
    for i in (0, 1, 500, 1999):
        b = bytearray(img)
        b[offs[i]] = 7
        check(sim, b, 256)
        check(sim, b, 4096)
    # garbage after a bad byte that still parses as records (a torn write):
    # the chain ends at the bad byte, the segments after it do not matter
    b = bytearray(img)
    b[offs[700]] = 0
    check(sim, b, 512)


def test_start_offsets(sim):
    rng = np.random.default_rng(13)
    img = random_log(rng, 1500)
    offs = chain(bytes(img))[0]
    for st in (offs[1], offs[777], offs[-1], len(img)):
        check(sim, img, 512, start=st)


def test_framed_records_inside_values(sim):
    """Values that are themselves WAL images (a log of logs): inside them the
    guesses find plausible chains that are not the log's.  The check catches
    each one; repairs keep the chain exact, and past wal_seg_rounds the walk
    declines (the caller then takes candidate doubling)."""
    rng = np.random.default_rng(14)
    inner = bytes(random_log(rng, 60, hi=120))
    parts = []
    for i in range(200):
        parts.append(rec(b"k%d" % i, inner if i % 3 == 0 else rng.bytes(int(rng.integers(0, 300)))))
    img = bytearray(b"".join(parts))
    for S in (256, 1024, 8192):
        rep = check(sim, img, S, rounds=1024)
        assert rep is not None
    # with no repairs allowed it declines rather than return a wrong chain
    assert sim(img, 256, rounds=0) is None or check(sim, img, 256, rounds=0) == 0


def test_type_byte_flood(sim):
    """Keys and values of 0x01 bytes: every byte a candidate, every false
    start a long plausible chain."""
    img = bytearray(b"".join(rec(b"\x01" * 40, b"\x01" * 200) for _ in range(300)))
    for S in (64, 512, 4096):
        check(sim, img, S, rounds=1024)
    img2 = bytearray(b"".join(rec(b"\x02" * 3, b"\x01\x00\x00\x00" * 50) for _ in range(300)))
    check(sim, img2, 512, rounds=1024)


def test_tiny_logs(sim):
    for img in (b"", b"\x01", b"\x02", b"\x05", rec(b""), rec(b"", b""), rec(b"a", b"b")[:-1],
                rec(b"key", b"value") + b"\x01\x00", rec(b"k") + b"\x09"):
        for S in (64, 4096):
            check(sim, bytearray(img), S)


def test_huge_lengths_wrap(sim):
    """klen + vlen wrapping in u32 (wal.rs:129), and a length past EOF."""
    r = struct.pack("<BIII", 1, 0, 0xFFFFFFF0, 0x20) + b"x" * 16  # wraps to 16
    img = bytearray(r * 50 + struct.pack("<BIII", 1, 0, 5, 1 << 30) + b"abc")
    for S in (64, 200):
        check(sim, img, S)


@pytest.mark.parametrize("S", [64, 512, 4096])
@pytest.mark.parametrize("parts", [2, 5, 17])
def test_prefix_walks_chain_to_the_whole(sim, S, parts):
    """The walk in prefixes (lim < n: the records that start before lim, and
    the first record start at or past lim as the next prefix's start), as the
    pipelined device replay runs it: the prefixes' records in order are the
    whole chain's, whatever the cut points -- inside headers, payloads, long
    records that cross several prefixes -- and the chain's end (clean EOF,
    truncated tail, bad type byte) lands in the right prefix."""
    rng = np.random.default_rng(S * 31 + parts)
    img = bytearray(random_log(rng, 3000, hi=900))
    for variant in range(3):
        im = bytes(img)
        if variant == 1:
            im = im[:len(im) - 7]  # EOF inside a payload or a header
        if variant == 2:
            want, _, _ = chain(im)
            b = bytearray(im)
            b[want[2222]] = 0x77  # bad type byte
            im = bytes(b)
        want = chain(im)
        n = len(im)
        cuts = sorted(set(int(c) for c in rng.integers(1, n, size=parts - 1)))
        r, got, end = 0, [], None
        for lim in cuts + [n]:
            if lim <= r:
                continue
            res = sim.prefix(im, r, lim, S)
            assert res is not None
            offs, code, pos = res
            assert all(r <= o < lim for o in offs)
            got += offs
            if code != 1:  # the chain ended in this prefix
                end = (code, pos if code == BAD else 0)
                break
            assert pos >= lim
            r = pos
        if end is None:  # the last prefix stopped exactly at n
            assert r >= n
            end = (END, 0)
        assert got == want[0]
        assert end == (want[1], want[2])


@pytest.mark.parametrize("stage", [0, 1, 6, 100000])
@pytest.mark.parametrize("nsub", [2, 4, 32])
@pytest.mark.parametrize("S", [256, 4096, 65536])
def test_emit_by_sub_segments(sim, S, nsub, stage):
    """The emit from the walk's checkpoints, one thread per sub-segment: the
    same records as the chain walk -- records longer than sub-segments and
    segments, entries after a sub-segment start, repairs (which rewalk and
    re-note the checkpoints), a bad type byte and a cut inside a record.
    stage: the walk's staging slots per segment (seg::StageRec) -- segments
    that fit are placed from their slots, the rest emitted, mixed in one walk."""
    sim.set_nsub(nsub)
    sim.set_stage(stage)
    try:
        rng = np.random.default_rng(S * 3 + nsub)
        for img in (random_log(rng, 1500, hi=900), random_log(rng, 200, lo=1000, hi=30000),
                    random_log(rng, 3000, hi=30)):
            check(sim, img, S)  # (asserts the records, the code and the bad byte)
            check(sim, img, S, start=1, shift=3)
            want, _, _ = chain(img)
            b = bytearray(img)
            b[want[len(want) // 2]] = 0x55
            check(sim, bytes(b), S)
            check(sim, img[:len(img) - 11], S)
    finally:
        sim.set_nsub(1)
        sim.set_stage(0)


def _mulmod(a, b):
    """a(x) * b(x) mod P(x), reflected (zlib's multmodp)."""
    m, p = 1 << 31, 0
    while True:
        if a & m:
            p ^= b
            if (a & (m - 1)) == 0:
                return p
        m >>= 1
        b = (b >> 1) ^ 0xEDB88320 if b & 1 else b >> 1


def test_unpack_constants():
    """unpack_crc's constants are x^-72 and x^-104 mod P(x): times x^72
    (x^104) they give x^0; pack_crc's are x^104 and x^72."""
    x8inv = 0x6567cb95  # x^-8: times x^8 (bit 23) is x^0 (bit 31)
    assert _mulmod(x8inv, 1 << 23) == 1 << 31
    r = 1 << 31
    pw = {}
    for k in range(1, 14):
        r = _mulmod(r, x8inv)
        pw[k] = r
    assert pw[9] == 0x2fb98a7d and pw[13] == 0x525983aa
    x8 = 1 << 23
    r = 1 << 31
    for k in range(1, 14):
        r = _mulmod(r, x8)
        if k == 9:
            assert r == 0x1eb014d8
    assert r == 0xe6050901


@pytest.mark.parametrize("stage", [0, 3, 100000])
@pytest.mark.parametrize("nsub", [1, 4])
@pytest.mark.parametrize("S", [512, 4096, 65536])
def test_packed_crc_spans(sim, S, nsub, stage):
    """The emit's packed CRC spans: record i's span is its payload and the next
    record's header (the last one's its payload alone), so the spans tile the
    log; seg::unpack_crc (wal_compare_packed's) takes the header back out of
    the span's CRC (zlib's here) to the payload's own, and so does the
    restatement of the algebra in Python."""
    import zlib
    M = 0xFFFFFFFF
    sim.set_nsub(nsub)
    sim.set_stage(stage)
    try:
        rng = np.random.default_rng(S + nsub)
        for img in (random_log(rng, 1500, hi=900), random_log(rng, 300, lo=1000, hi=30000),
                    random_log(rng, 2000, hi=30, remove_every=3)):
            cut = bytearray(img[:len(img) - 7])
            bad = bytearray(img)
            want0, _, _ = chain(img)
            bad[want0[len(want0) // 2]] = 0x55
            for im in (img, bytes(cut), bytes(bad)):
                offs, _, _ = chain(im)
                po, pl, pe = sim.packed(im, S)
                assert len(po) == len(offs)
                for i, q in enumerate(offs):
                    hl = 13 if im[q] == 1 else 9
                    klen, vlen = struct.unpack_from("<II", im, q + 5)
                    if hl == 9:
                        vlen = 0
                    plen = min((klen + vlen) & M, len(im) - q - hl)
                    assert po[i] == q + hl
                    span = zlib.crc32(im[po[i]:po[i] + pl[i]])
                    stored = struct.unpack_from("<I", im, q + 1)[0]
                    if i + 1 < len(offs):  # pack_crc: the stored CRC carried over the next header
                        nq = offs[i + 1]
                        nh = 13 if im[nq] == 1 else 9
                        g = ~zlib.crc32(im[nq:nq + nh], M) & M
                        want = ~(_mulmod(~stored & M, 0xe6050901 if nh == 13 else 0x1eb014d8) ^ g) & M
                        assert pe[i] == want, i
                        # ... which is the span's CRC exactly when the stored one is the payload's
                        pay = zlib.crc32(im[q + hl:q + hl + plen])
                        assert ~(_mulmod(~pay & M, 0xe6050901 if nh == 13 else 0x1eb014d8) ^ g) & M == span
                    else:
                        assert pe[i] == stored
                    if i + 1 < len(offs):
                        nq = offs[i + 1]
                        nh = 13 if im[nq] == 1 else 9
                        assert po[i] + pl[i] == nq + nh
                        t, crc, k2 = struct.unpack_from("<BII", im, nq)
                        v2 = struct.unpack_from("<I", im, nq + 9)[0] if nh == 13 else 0
                        got = sim.unpack(span, t, crc, k2, v2)
                        g = ~zlib.crc32(im[nq:nq + nh], M) & M
                        alg = ~_mulmod(~span & M ^ g, 0x525983aa if nh == 13 else 0x2fb98a7d) & M
                        assert got == alg == zlib.crc32(im[q + hl:q + hl + plen]), i
                    else:
                        assert pl[i] == plen and span == zlib.crc32(im[q + hl:q + hl + plen])
    finally:
        sim.set_nsub(1)
        sim.set_stage(0)


def test_log_of_logs_parallel_repair(sim):
    """Values that are WAL images, each shorter than a segment: every
    segment's guess lies inside a value and follows the value's own chain,
    which ends at the log's next header -- every guess is wrong, every walk's
    exit right.  One parallel repair round (seg_prepair: each segment walked
    again from its predecessor's exit, all at once) makes the chain exact with
    no serial repair; without it the serial repair walks segment after
    segment."""
    rng = np.random.default_rng(21)
    parts = []
    for i in range(400):
        inner = bytes(random_log(rng, int(rng.integers(4, 12)), lo=20, hi=150))
        parts.append(rec(b"v%d" % i, inner))
    img = bytearray(b"".join(parts))
    for S in (2048, 4096, 8192):
        try:
            sim.set_prepair(2)
            assert check(sim, img, S, rounds=0) == 0  # no serial repair needed
            assert sim.prepairs() >= 1
            sim.set_prepair(0)
            rep = check(sim, img, S, rounds=1 << 20)
            assert rep >= 1 and sim.prepairs() == 0
        finally:
            sim.set_prepair(2)


@pytest.mark.parametrize("prepair", [0, 1, 2, 8])
def test_parallel_repair_keeps_every_chain(sim, prepair):
    """The parallel round is only a proposal the check verifies: with 0 to 8
    rounds allowed, adversarial logs (long records over tiny segments, type
    byte floods, framed values, cuts) give the plain chain walk's records."""
    rng = np.random.default_rng(22 + prepair)
    try:
        sim.set_prepair(prepair)
        img = random_log(rng, 800)
        for S in (64, 300, 4096):
            check(sim, img, S, rounds=1 << 20)
        parts = [rec(rng.bytes(8), rng.bytes(int(L))) for L in rng.integers(0, 20000, 120)]
        check(sim, bytearray(b"".join(parts)), 1000, rounds=1 << 20)
        flood = bytearray(b"".join(rec(b"\x01" * 40, b"\x01" * 200) for _ in range(150)))
        check(sim, flood, 512, rounds=1 << 20)
        inner = bytes(random_log(rng, 60, hi=120))
        lol = bytearray(b"".join(rec(b"k%d" % i, inner if i % 3 == 0 else rng.bytes(int(rng.integers(0, 300))))
                                 for i in range(150)))
        for S in (256, 1024):
            check(sim, lol, S, rounds=1 << 20)
        for cut in range(0, len(lol), 997):
            check(sim, lol[:cut], 512, rounds=1 << 20)
    finally:
        sim.set_prepair(2)


def test_first_records_past_the_later_rule(sim):
    """Segments of 512 KiB - 1 MiB over records of 300-900 KiB: every true
    first record is longer than kLaterMax, so the later-start rule is skipped
    for it; a wrong guess it would have refused is caught by the check.  The
    plain chain either way, with and without the parallel rounds."""
    rng = np.random.default_rng(23)
    img = bytearray(b"".join(rec(rng.bytes(16), rng.bytes(int(L))) for L in rng.integers(300 << 10, 900 << 10, 60)))
    for prepair in (2, 0):
        try:
            sim.set_prepair(prepair)
            for S in (512 << 10, 1 << 20):
                check(sim, img, S, rounds=1 << 20)
        finally:
            sim.set_prepair(2)
