"""The walking CRC kernel's record map (crc32_walk_kernel, lsmck_crc32.hip),
simulated lane by lane on the host (tools/walk_sim.py): every valid lane maps
to the segment a plain enumeration gives, reads only its own record, and every
record is emitted exactly once.  CPU-only; the GPU tests check the CRCs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import walk_sim  # noqa: E402


def test_walk_map_random_batches():
    rng = np.random.default_rng(7)
    for tr in range(12):
        n = int(rng.integers(1, 2500))
        kind = tr % 4
        if kind == 0:
            lens = rng.integers(0, 700, n)
        elif kind == 1:
            lens = rng.integers(0, 130, n)
        elif kind == 2:
            lens = rng.integers(0, 300, n)
            lens[rng.integers(0, n, 2)] = rng.integers(1 << 15, 1 << 19, 2)
        else:
            lens = np.zeros(n, dtype=np.int64)
        walk_sim.simulate(np.asarray(lens, dtype=np.int64), int(rng.choice([1, 5, 64])))


def test_walk_map_edges():
    for lens in ([0], [1], [128], [129], [128 * 64], [128 * 64 + 1], [8192 * 3 - 1] * 5, [64] * 1000):
        walk_sim.simulate(np.asarray(lens, dtype=np.int64), 3)
