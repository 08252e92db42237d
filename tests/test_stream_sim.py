"""The algebra of the stream kernel (crc32_stream_kernel, lsmck_crc32.hip),
as modelled lane by lane in tools/stream_sim.py, against zlib: register resets
at record boundaries, the exact boundary capture, the Horner carry inside and
across tiles, and the per-record finish.  CPU only (the GPU parity tests are
tests/test_gpu_stream.py)."""
import os
import random
import sys
import zlib

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import stream_sim  # noqa: E402


@pytest.mark.parametrize("lens_kind", ["min", "mixed", "grid"])
def test_stream_model_matches_zlib(lens_kind):
    rnd = random.Random(lens_kind)
    if lens_kind == "min":
        lens = [64] * 150  # two boundaries in half the chunks
    elif lens_kind == "grid":
        lens = [128] * 70 + [192, 64] * 20  # boundaries at chunk byte 0 and at a chain start
    else:
        lens = [rnd.choice([64, 65, 67, 100, 127, 129, 191, 255, 300, 1000, 9000]) for _ in range(60)]
    lead = 0 if lens_kind == "grid" else rnd.randrange(128)
    starts, p = [], lead
    for ln in lens:
        starts.append(p)
        p += ln
    data = bytes(rnd.randrange(256) for _ in range(p + 64))
    got = stream_sim.simulate(data, starts, p)
    assert got == [zlib.crc32(data[s:s + ln]) for s, ln in zip(starts, lens)]
