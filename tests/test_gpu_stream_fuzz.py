"""Randomised batches through the stream kernel (crc32_stream_kernel,
lsmck_crc32.hip) against the oracle (crc 1.x's algorithm, oracle/lsmck_oracle.c),
round 6: after the per-chain event bodies and the bank-aware Horner tables,
each seed draws its own mix -- record lengths from several distributions at
once (64 B records that put two boundaries in a chunk, lengths around the
128-byte chunk and 8 KiB tile edges, long records over several tiles), gaps
of 0..64 bytes as a WAL's headers leave (some seeds packed), a random lead
and a random misalignment of the data in its allocation.  The stream kernel
alone (crc_stream 2: a declined batch would leave the outputs unwritten)."""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

EDGES = [64, 65, 66, 67, 68, 95, 96, 97, 127, 128, 129, 130, 131, 132, 191, 192, 193, 255, 256, 257,
         4095, 4096, 4097, 8063, 8064, 8127, 8128, 8129, 8191, 8192, 8193, 8256, 16383, 16384, 16385]


def _batch(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2000, 12000))
    kinds = rng.choice(4, size=n, p=rng.dirichlet([1.0, 1.0, 1.0, 0.3]))
    lens = np.empty(n, dtype=np.uint32)
    for k, pick in ((0, lambda m: np.full(m, 64)),
                    (1, lambda m: rng.choice(EDGES, m)),
                    (2, lambda m: rng.integers(64, 3000, m)),
                    (3, lambda m: rng.integers(8000, 70000, m))):
        idx = np.nonzero(kinds == k)[0]
        lens[idx] = pick(len(idx))
    packed = rng.random() < 0.4
    gaps = np.zeros(n, dtype=np.uint64) if packed else rng.choice([0, 9, 13, 13, 13, 64], n).astype(np.uint64)
    lead = int(rng.integers(0, 400))
    step = gaps + np.concatenate([[0], lens[:-1]]).astype(np.uint64)
    off = np.cumsum(step) + np.uint64(lead)
    shift = int(rng.integers(0, 4))
    return off, lens, shift


@pytest.mark.parametrize("seed", list(range(24)))
def test_random_batches_vs_oracle(ctx, seed):
    off, ln, shift = _batch(zlib.crc32(f"stream-fuzz-{seed}".encode()))
    n = len(off)
    size = int(off[-1]) + int(ln[-1]) + 16
    data = O.gen_stream(0x5F0220 + seed, 0, size)
    want = O.crc32_batch(data, off, ln, threads=8)
    d = ctx.alloc(size + shift)
    d.upload(data, offset=shift)
    d_o, d_l, out = ctx.alloc(8 * n), ctx.alloc(4 * n), ctx.alloc(4 * n)
    out.upload(np.full(n, 0xA5A5A5A5, dtype=np.uint32))
    d_o.upload(off)
    d_l.upload(ln)
    ctx.set_option("crc_stream", 2)
    try:
        ctx.crc32_device(d.ptr + shift, d_o.ptr, d_l.ptr, n, out.ptr)
        ctx.sync()
    finally:
        ctx.set_option("crc_stream", 1)
    got = out.download(np.uint32)
    for b in (d, d_o, d_l, out):
        b.free()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (seed, n, bad[:8].tolist(), ln[bad[:8]].tolist())
