#!/usr/bin/env python3
"""LDS bank-conflict model of the stream kernel's table lookups
(lsmck_crc32.hip), per 8 KiB tile: extra LDS cycles of each ds_read_b32 as
MI355X_MICROARCH.md "LDS" states them -- two 32-lane groups, bank = (address
/ 4) mod 32, each extra distinct address on a bank adds a cycle; equal
addresses broadcast.

Covers the lookups whose addresses depend on data: the bulk chains (the 32x
replicated slicing tables), shift_bytes32<2> (plain tables) and the Horner
shift's two nibble stages, in the round-6 first layout ([j][q][b] /
[G][q][j'][a]) and the bank-aware one ([j][q][f] / [j][h][q], d = 16h + f).
Lane d's: a tile without events shifts lane l by 63 - l; an event tile by
the distance to the chunk before the next record end (5 ends a tile here,
config 3's mean).

Checked against the counters: SQ_LDS_BANK_CONFLICT of the bulk-only
ablation (crc_ablate 10) is 78.6 extra cycles per tile (profiles/r06/lds/),
this model 81.2 for the first layout.
  python3 tools/lds_conflicts.py"""
import random

COLS = 131072 + 12288


def extra_cycles(addrs):
    ex = 0
    for g in (addrs[:32], addrs[32:]):
        banks = {}
        for a in g:
            banks.setdefault((a // 4) % 32, set()).add(a)
        ex += max(len(s) for s in banks.values()) - 1
    return ex


def horner_first(v, u, d, j):
    """round 6's first layout: stage 1 [j][q][b] (b = d & 3), stage 2 [G][q][j'][a] (a = d >> 2)"""
    n1, n2 = COLS + 8192, COLS
    a1 = n1 + 256 * j + 16 * ((v >> (4 * j)) & 15) + 4 * (d & 3)
    a2 = n2 + 4096 * (j >> 2) + 256 * ((u >> (4 * j)) & 15) + 64 * (j & 3) + 4 * (d >> 2)
    return a1, a2


def horner_bank(v, u, d, j):
    """the bank-aware layout: stage A [j][q][f] (f = d & 15), stage B [j][h][q] (h = d >> 4)"""
    na, nb = COLS, COLS + 8192
    a1 = na + 1024 * j + 64 * ((v >> (4 * j)) & 15) + 4 * (d & 15)
    a2 = nb + 256 * j + 64 * (d >> 4) + 4 * ((u >> (4 * j)) & 15)
    return a1, a2


def lane_d(kind, rng, ends=5):
    if kind == "bulk":
        return [63 - lane for lane in range(64)]
    e = sorted(rng.sample(range(64), ends))
    out = []
    for lane in range(64):
        above = [c for c in e if c > lane]
        out.append((above[0] if above else 64) - 1 - lane)
    return out


def horner_cycles(layout, kind, tiles=500, seed=1):
    rng = random.Random(seed)
    s1 = s2 = 0
    for _ in range(tiles):
        ds = lane_d(kind, rng)
        vs = [rng.getrandbits(32) for _ in range(64)]
        us = [rng.getrandbits(32) for _ in range(64)]
        for j in range(8):
            a = [layout(vs[lane], us[lane], ds[lane], j) for lane in range(64)]
            s1 += extra_cycles([x[0] for x in a])
            s2 += extra_cycles([x[1] for x in a])
    return s1 / tiles, s2 / tiles


def other_cycles(tiles=500, seed=1):
    """bulk chains (per lookup) and shift_bytes32<2> (per tile)"""
    rng = random.Random(seed)
    bulk = sum(extra_cycles([256 * rng.randrange(256) + 4 * (lane % 32) + 128 for lane in range(64)])
               for _ in range(tiles)) / tiles
    sh = 0
    for _ in range(tiles):
        vs = [rng.getrandbits(32) for _ in range(64)]
        for k in range(4):
            sh += extra_cycles([131072 + 4096 + 1024 * k + 4 * ((vs[lane] >> (8 * k)) & 255) for lane in range(64)])
    return bulk, sh / tiles


def main():
    bulk, sh = other_cycles()
    print(f"bulk chain lookup: {bulk:.1f} extra cycles each; shift_bytes32<2>: {sh:.1f} per tile")
    for name, lay in (("first layout", horner_first), ("bank-aware layout", horner_bank)):
        for kind in ("bulk", "event"):
            a, b = horner_cycles(lay, kind)
            print(f"Horner, {name}, {kind} tile: stage 1 {a:.1f} + stage 2 {b:.1f} = {a + b:.1f} extra cycles")


if __name__ == "__main__":
    main()
