"""Host model of the stream kernel's Horner shift by nibble tables
(lsmck_crc32.hip: build_nib / nib_mul, round 6, the bank-aware layout
d = 16h + f): the tables are laid out in a
model of the LDS at the kernel's byte addresses, each lookup's address is
formed exactly as the kernel forms it (one OR of the shifted value's nibble
with a per-lane base, plus the instruction's immediate offset), and the result
must equal the direct GF(2) product v (x) x^(8*128*d) for every d = 0..63.
This pins the layout (alignments, strides, the or-addressing) on the CPU; the
GPU tests check the kernel's CRCs against the oracle."""
import random

POLY = 0xEDB88320
LDS_COLS_OFF = 131072 + 12288  # LDS_SHIFT_OFF + LDS_SHIFT_BYTES
NA = LDS_COLS_OFF          # LDS_NIBA_OFF: [8 j][16 q][16 f]
NB = LDS_COLS_OFF + 8192   # LDS_NIBB_OFF: [8 j][4 h][16 q]
KLO = LDS_COLS_OFF + 8192 + 2048  # LDS_KLO_OFF (COLS 8 KiB + KHI 2 KiB)


def gf2_mulmod(a, b):
    """lsmck_crc32.hip gf2_mulmod (zlib multmodp): a (x) b, reflected."""
    p = 0
    for i in range(32):
        if (a << i) & 0x80000000:
            p ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return p & 0xFFFFFFFF


def x_pow(n):
    r = 0x80000000  # x^0
    for _ in range(n):
        r = (r >> 1) ^ (POLY if r & 1 else 0)
    return r


KSEG = [0x80000000]
K1 = x_pow(8 * 128)
for _ in range(63):
    KSEG.append(gf2_mulmod(KSEG[-1], K1))


def build(lds):
    for i in range(2560):
        if i < 2048:
            f, q, j = i & 15, (i >> 4) & 15, i >> 8
            e = f
            addr = NA + 1024 * j + 64 * q + 4 * f
        else:
            k = i - 2048
            q, h, j = k & 15, (k >> 4) & 3, k >> 6
            e = 16 * h
            addr = NB + 256 * j + 64 * h + 4 * q
        assert addr not in lds
        lds[addr] = gf2_mulmod((q << (4 * j)) & 0xFFFFFFFF, KSEG[e])


def sh(v, s):
    """v shifted right by s (left by -s), 32 bits"""
    return (v >> s) if s >= 0 else (v << -s) & 0xFFFFFFFF


def nib_mul(lds, v, d):
    bA = NA + ((d & 15) << 2)
    bB = NB + ((d >> 4) << 6)
    u = 0
    for j in range(8):  # stage A: nibble j at bits 6-9 of v >> (4j - 6), row j by the immediate
        u ^= lds[((sh(v, 4 * j - 6) & 0x3C0) | bA) + 1024 * j]
    y = 0
    for j in range(8):  # stage B: nibble j at bits 2-5 of u >> (4j - 2)
        y ^= lds[((sh(u, 4 * j - 2) & 0x3C) | bB) + 256 * j]
    return y


def test_layout_fits_between_the_shift_tables_and_klo():
    lds = {}
    build(lds)
    assert min(lds) == LDS_COLS_OFF and max(lds) + 4 == KLO  # COLS + KHI exactly, nothing over klo
    assert NA & 0x3FC == 0 and NB & 0xFC == 0  # the or-addressing's index bits are clear in the bases


def test_nib_mul_equals_the_gf2_product():
    lds = {}
    build(lds)
    rng = random.Random(6)
    vals = [0, 1, 0x80000000, 0xFFFFFFFF, 0x12345678] + [rng.getrandbits(32) for _ in range(60)]
    for d in range(64):
        for v in vals:
            assert nib_mul(lds, v, d) == gf2_mulmod(v, KSEG[d]), (hex(v), d)


def test_layout_bank_conflicts_model():
    """The bank-aware layout against round 6's first one, in the LDS model of
    tools/lds_conflicts.py (ds_read_b32: two 32-lane groups, bank = address/4
    mod 32): a Horner without events conflicts only in stage A (lanes l and
    l + 16 share f), and an event tile's Horner a quarter as much as before."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "lds_conflicts", os.path.join(os.path.dirname(__file__), "..", "tools", "lds_conflicts.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    # the model's addresses are the kernel's (the same bases as build() above)
    assert m.horner_bank(0x12345678, 0, 37, 3)[0] == NA + 1024 * 3 + 64 * 5 + 4 * (37 & 15)
    assert m.horner_bank(0, 0x9ABCDEF0, 37, 5)[1] == NB + 256 * 5 + 64 * (37 >> 4) + 4 * 0xB
    a1, b1 = m.horner_cycles(m.horner_bank, "bulk", tiles=60)
    assert b1 == 0.0 and a1 <= 16.0
    fa, fb = m.horner_cycles(m.horner_first, "bulk", tiles=60)
    assert fa + fb >= 3 * (a1 + b1)
    ea, eb = m.horner_cycles(m.horner_bank, "event", tiles=60)
    ga, gb = m.horner_cycles(m.horner_first, "event", tiles=60)
    assert ga + gb >= 3 * (ea + eb)
