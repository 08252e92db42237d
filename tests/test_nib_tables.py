"""Host model of the stream kernel's Horner shift by nibble tables
(lsmck_crc32.hip: build_nib / nib_mul, round 6): the tables are laid out in a
model of the LDS at the kernel's byte addresses, each lookup's address is
formed exactly as the kernel forms it (one OR of the shifted value's nibble
with a per-lane base, plus the instruction's immediate offset), and the result
must equal the direct GF(2) product v (x) x^(8*128*d) for every d = 0..63.
This pins the layout (alignments, strides, the or-addressing) on the CPU; the
GPU tests check the kernel's CRCs against the oracle."""
import random

POLY = 0xEDB88320
LDS_COLS_OFF = 131072 + 12288  # LDS_SHIFT_OFF + LDS_SHIFT_BYTES
NIB2 = LDS_COLS_OFF
NIB1 = LDS_COLS_OFF + 8192
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
        if i < 512:
            b = i & 3
            q = (i >> 2) & 15
            j = i >> 6
            e = b
            addr = NIB1 + 256 * j + 16 * q + 4 * b
        else:
            k = i - 512
            a, jp, g = k & 15, (k >> 4) & 3, k >> 10
            q = (k >> 6) & 15
            j = 4 * g + jp
            e = 4 * a
            addr = NIB2 + 4096 * g + 256 * q + 64 * jp + 4 * a
        assert addr not in lds
        lds[addr] = gf2_mulmod((q << (4 * j)) & 0xFFFFFFFF, KSEG[e])


def nib_mul(lds, v, d):
    m = 0xFFFFFFFF
    b1 = NIB1 + ((d & 3) << 2)
    b2 = NIB2 + (d & ~3)
    ld = lambda a: lds[a]  # noqa: E731
    st1 = [((v << 4) & 0xF0) | b1, ((v & 0xF0) | b1) + 256, (((v >> 4) & 0xF0) | b1) + 512,
           (((v >> 8) & 0xF0) | b1) + 768, (((v >> 12) & 0xF0) | b1) + 1024, (((v >> 16) & 0xF0) | b1) + 1280,
           (((v >> 20) & 0xF0) | b1) + 1536, (((v >> 24) & 0xF0) | b1) + 1792]
    u = 0
    for a in st1:
        u ^= ld(a)
    st2 = [(((u << 8) & m) & 0xF00) | b2, ((((u << 4) & m) & 0xF00) | b2) + 64, ((u & 0xF00) | b2) + 128,
           (((u >> 4) & 0xF00) | b2) + 192, (((u >> 8) & 0xF00) | b2) + 4096, (((u >> 12) & 0xF00) | b2) + 4160,
           (((u >> 16) & 0xF00) | b2) + 4224, (((u >> 20) & 0xF00) | b2) + 4288]
    y = 0
    for a in st2:
        y ^= ld(a)
    return y


def test_layout_fits_between_the_shift_tables_and_klo():
    lds = {}
    build(lds)
    assert min(lds) == LDS_COLS_OFF and max(lds) + 4 == KLO  # COLS + KHI exactly, nothing over klo
    assert NIB2 % 4096 == 0 and NIB1 % 256 == 0


def test_nib_mul_equals_the_gf2_product():
    lds = {}
    build(lds)
    rng = random.Random(6)
    vals = [0, 1, 0x80000000, 0xFFFFFFFF, 0x12345678] + [rng.getrandbits(32) for _ in range(60)]
    for d in range(64):
        for v in vals:
            assert nib_mul(lds, v, d) == gf2_mulmod(v, KSEG[d]), (hex(v), d)
