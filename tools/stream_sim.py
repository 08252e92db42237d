#!/usr/bin/env python3
"""Lane-level simulator of crc32_stream_kernel (lsmck_crc32.hip): the CRC-32s
of packed records of >= 64 bytes computed from aligned 128-byte chunks of the
byte stream, exactly as the kernel's lanes and waves do it, checked against
zlib.  Run it after any change to the kernel's algebra:

  python3 tools/stream_sim.py [--records N] [--seed S]

Model (all values are raw CRC registers; (x) is the product mod P):
  * chunk = 32 little-endian words in two chains of 16; a chain's register
    starts at 0; F(v) = v (x) x^32 is one word step.
  * a record boundary at chunk byte j lies in chain h = j >= 64, word w = j/4,
    t = j % 4, mlo = the mask of the word's t bytes before j.  The chain's
    register after that word is RESET to F(~(u_w | mlo)) ^ mlo: the new
    record's bytes from j with the 0xFFFFFFFF init folded in (no dependency on
    the chain's register).  The capture A' = the register c advanced over the
    t bytes before j, = (c >> 8t) ^ XOR_{i<t} T_{t-1-i}[(c ^ u_w) byte i]
    (slicing-by-t; the kernel saves c ^ u_w and u_w at the boundary word and
    runs the t lookups once after the chunk).
  * a chunk's tail T = the register of its last piece aligned to the chunk end
    (chain 1 alone if it holds a boundary, else shift64(R0) ^ R1).
  * per lane G = T (x) x^(1024 d), d = (next boundary chunk in the tile) - 1 -
    lane; X = prefix XOR of G over the wave; the record ending at chunk c
    (started at chunk ls in this tile, or before it) has Hprev = X[c-1] ^
    X[ls-1] (or ^ carry (x) x^(1024 c)).
  * its CRC = ~(P (x) x^(8m) ^ A'), P = Hprev for a chain-0 end,
    shift64(Hprev) ^ R0 for a chain-1 end, m = j - 64h.
"""
import argparse
import random
import zlib

POLY = 0xEDB88320
ONE = 0x80000000


def mul(a, b):
    """multmodp: reflected GF(2)[x] product mod P."""
    m, p = 1 << 31, 0
    while a:
        if a & m:
            p ^= b
            a ^= m
        m >>= 1
        b = (b >> 1) ^ POLY if b & 1 else b >> 1
    return p


def xpow(k):
    r, base = ONE, 0x40000000
    while k:
        if k & 1:
            r = mul(r, base)
        base = mul(base, base)
        k >>= 1
    return r


ORD = (1 << 32) - 1
X32 = xpow(32)
X512 = xpow(512)


def F(v):
    return mul(v, X32)


def _tables():
    t0 = []
    for n in range(256):
        c = n
        for _ in range(8):
            c = (c >> 1) ^ POLY if c & 1 else c >> 1
        t0.append(c)
    tabs = [t0]
    for _ in range(3):
        prev = tabs[-1]
        tabs.append([(v >> 8) ^ t0[v & 0xFF] for v in prev])
    return tabs


TAB = _tables()  # slicing-by-4 tables: T_k[n] = T0[n] advanced over k zero bytes


def chunk_lane(words, bounds):
    """One lane: 32 words, its boundaries (<= 1 per chain, chunk bytes j).
    Returns (R0, R1, cap0, cap1, tail)."""
    jc = [None, None]
    for j in bounds:
        jc[1 if j >= 64 else 0] = j
    R, cap = [0, 0], [0, 0]
    for h in (0, 1):
        c = 0
        for k in range(16):
            w = 16 * h + k
            u = words[w]
            x = c ^ u
            if jc[h] is not None and (jc[h] >> 2) == w:
                t = jc[h] & 3
                mlo = (1 << (8 * t)) - 1  # keep the low t bytes (little endian)
                # the capture: t byte steps of the register c over the word's
                # bytes before j, as slicing-by-t from the saved x = c ^ u
                ax = c >> (8 * t)
                for i in range(t):
                    ax ^= TAB[t - 1 - i][(x >> (8 * i)) & 0xFF]
                cap[h] = ax
                # the reset: the register after the word for a record starting
                # at byte t, init included, = F(~(u | mlo)) ^ mlo (no c in it)
                c = F(~(u | mlo) & 0xFFFFFFFF) ^ mlo
                continue
            c = F(x)
        R[h] = c
    tail = R[1] if jc[1] is not None else (mul(R[0], X512) ^ R[1])
    return R[0], R[1], cap[0], cap[1], tail


def simulate(data, starts, dend, tiles_per_wave=3):
    """data: the packed stream from byte A0 (= 0 here, 128-aligned) on;
    starts: record start offsets; dend: end of the last record."""
    n = len(starts)
    pos = list(starts) + [dend]  # boundary b: the start of record b (b = n: the end)
    nchunk = (dend >> 7) + 1
    ntiles = (nchunk + 63) // 64
    out = [None] * n
    buf = data + bytes(ntiles * 8192 - len(data))
    carry = None  # value of the record crossing the tile boundary (aligned to the tile's end)
    bt = 0
    for t in range(ntiles):
        T0 = 8192 * t
        cnt = 0
        while bt + cnt <= n and pos[bt + cnt] < T0 + 8192:
            cnt += 1
        assert cnt <= 128
        bs = [(pos[bt + i] - T0) for i in range(cnt)]  # tile-relative boundaries, sorted
        lane_b = [[] for _ in range(64)]
        for r in bs:
            lane_b[r >> 7].append(r & 127)
        L = []
        for l in range(64):
            off = T0 + 128 * l
            ws = [int.from_bytes(buf[off + 4 * i:off + 4 * i + 4], "little") for i in range(32)]
            L.append(chunk_lane(ws, lane_b[l]))
        # Horner inside the tile
        G = []
        for l in range(64):
            nxt = next((c for c in range(l + 1, 64) if lane_b[c]), 64)
            d = nxt - 1 - l
            G.append(mul(L[l][4], xpow(1024 * d)))
        X, acc = [], 0
        for g in G:
            acc ^= g
            X.append(acc)
        Xm = lambda c: X[c - 1] if c >= 1 else 0  # noqa: E731
        # record phase: window index i = boundary bt + i ends record bt + i - 1
        for i in range(cnt):
            r = bt + i - 1
            c, j = bs[i] >> 7, bs[i] & 127
            if i == 0:
                H = Xm(c) ^ (mul(carry, xpow(1024 * c)) if carry is not None else 0)
            else:
                H = Xm(c) ^ Xm(bs[i - 1] >> 7)
            h = 1 if j >= 64 else 0
            R0, R1, cap0, cap1, _ = L[c]
            A = cap1 if h else cap0
            P = mul(H, X512) ^ R0 if h else H
            m = j - 64 * h
            v = mul(P, xpow(8 * m)) ^ A
            if 0 <= r < n:
                out[r] = (~v) & 0xFFFFFFFF
        # carry out: the record active at the tile's end
        if cnt:
            ls = bs[-1] >> 7
            carry = X[63] ^ Xm(ls)
        else:
            carry = X[63] ^ (mul(carry, xpow(1024 * 64)) if carry is not None else 0)
        bt += cnt
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rnd = random.Random(a.seed)
    fails = 0
    for trial in range(6):
        lens = [rnd.choice([64, 65, 67, 100, 127, 128, 129, 191, 192, 255, 256, 300, 1000, 5000, 9000])
                for _ in range(a.records)]
        if trial == 0:
            lens = [64] * a.records  # two boundaries in many chunks
        lead = rnd.randrange(0, 128)
        starts, p = [], lead
        for ln in lens:
            starts.append(p)
            p += ln
        data = bytes(rnd.randrange(256) for _ in range(p + 64))
        got = simulate(data, starts, p)
        want = [zlib.crc32(data[s:s + ln]) for s, ln in zip(starts, lens)]
        bad = sum(1 for x, y in zip(got, want) if x != y)
        print(f"trial {trial}: lead {lead}, {len(lens)} records, {bad} mismatches")
        fails += bad
    raise SystemExit(1 if fails else 0)


if __name__ == "__main__":
    main()
