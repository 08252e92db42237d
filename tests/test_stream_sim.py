"""The algebra of the stream kernel (crc32_stream_kernel, lsmck_crc32.hip),
as modelled lane by lane in tools/stream_sim.py, against zlib: register resets
at record starts, the exact capture at record ends, gap bytes between records
(the WAL's headers) dropped by the resets, short records checksummed by their
window lane, the Horner carry inside and across tiles and wave cuts, and the
per-record finish.  CPU only (the GPU parity tests are
tests/test_gpu_stream.py)."""
import os
import random
import sys
import zlib

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import stream_sim  # noqa: E402


def _layout(lens, gaps, lead):
    offs, p = [], lead
    for ln, g in zip(lens, gaps):
        p += g
        offs.append(p)
        p += ln
    return offs, p


@pytest.mark.parametrize("kind", ["packed64", "mixed", "wal", "tiny"])
def test_stream_model_matches_zlib(kind):
    rnd = random.Random(kind)
    offs, lens, end = stream_sim.gen(rnd, 160, kind)
    data = bytes(rnd.randrange(256) for _ in range(end + 64))
    got = stream_sim.simulate(data, offs, lens, waves=3)
    assert got == [zlib.crc32(data[s:s + ln]) for s, ln in zip(offs, lens)]


@pytest.mark.parametrize("case", ["grid", "tile_edges", "gap_over_tile"])
def test_stream_model_edges(case):
    """Starts and ends on the 128-byte grid and at chain starts; ends exactly
    at a tile's end (the next tile's byte 0); a header gap across a tile edge."""
    rnd = random.Random(case)
    if case == "grid":
        lens = [128] * 70 + [192, 64] * 20
        gaps = [0] * len(lens)
        lead = 0
    elif case == "tile_edges":
        lens = [8192 - 13, 8192 - 9, 4096, 4096 - 13, 64, 8192] * 4
        gaps = [13, 9, 0, 13, 0, 0] * 4
        lead = 13
    else:
        lens = [8192 - 70, 100, 8192 - 5, 63, 64] * 5
        gaps = [13, 13, 9, 13, 0] * 5
        lead = 60
    offs, end = _layout(lens, gaps, lead)
    data = bytes(rnd.randrange(256) for _ in range(end + 64))
    for waves in (1, 4):
        got = stream_sim.simulate(data, offs, lens, waves=waves)
        assert got == [zlib.crc32(data[s:s + ln]) for s, ln in zip(offs, lens)]
