#!/usr/bin/env python3
"""Lane-level simulator of crc32_stream_kernel (lsmck_crc32.hip): the CRC-32s
of a batch of records that are sorted and do not overlap -- packed back to
back (config 3), or with gaps between them (a WAL image: the 13- or 9-byte
record header sits between two payloads) -- computed from aligned 128-byte
chunks of the byte stream, exactly as the kernel's lanes and waves do it, and
checked against zlib.  Run it after any change to the kernel's algebra:

  python3 tools/stream_sim.py [--records N] [--seed S]

Model (all values are raw CRC registers; (x) is the product mod P):
  * chunk = 32 little-endian words in two chains of 16; a chain's register
    starts at 0 (lane 0 of a tile: at the carry, below); F(v) = v (x) x^32 is
    one word step.
  * a LONG record (>= 64 bytes) has two events: its START and its END (the
    byte after its last).  A chain (64 bytes) holds at most one end and at
    most one start of long records, the end first.  At a start at chunk byte j
    (word w = j/4, t = j%4, mlo = the mask of the word's t bytes before j) the
    chain's register after the word is RESET to F(~(u_w | mlo)) ^ mlo: the new
    record's bytes from j with the 0xFFFFFFFF init folded in.  At an end the
    CAPTURE A' = the register c advanced over the word's t bytes before j,
    = (c >> 8t) ^ XOR_{i<t} T_{t-1-i}[(c ^ u_w) byte i].
  * a chunk's tail T = the register of its last piece aligned to the chunk end
    (chain 1 alone if chain 1 holds a start, else shift64(R0) ^ R1).
  * per lane G = T (x) x^(1024 d), d = (next chunk above the lane holding an
    END) - 1 - lane; X = prefix XOR of G over the wave; Y(c) = X[c-1] (0 for
    c = 0).
  * a long record ending at chunk c, byte j (chain h = j >= 64, m = j - 64h)
    and starting at chunk s of this tile has H = Y(c) ^ Y(s); one started in
    an earlier tile has H = Y(c) -- its raw value up to the tile start (the
    CARRY) entered lane 0's chain 0 as the initial register.  Its CRC =
    ~(P (x) x^(8m) ^ A'), P = H for a chain-0 end, shift64(H) ^ R0 for a
    chain-1 end.
  * the carry out of a tile: X[63] ^ Y(chunk of the tile's last start).
  * a SHORT record (< 64 bytes) has no events; the lane of the window that
    holds it checksums its bytes directly.
  * gap bytes between records are read and run through the chains like any
    other byte; the resets drop them.
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


def chunk_lane(words, ends, starts, init=0):
    """One lane: 32 words; its long-record events (chunk bytes; <= 1 end and
    <= 1 start per chain).  Returns (R0, R1, cap0, cap1, tail)."""
    je, js = [None, None], [None, None]
    for j in ends:
        assert je[j >> 6] is None
        je[j >> 6] = j
    for j in starts:
        assert js[j >> 6] is None
        js[j >> 6] = j
    R, cap = [0, 0], [0, 0]
    for h in (0, 1):
        if je[h] is not None and js[h] is not None:
            assert je[h] <= js[h]
        c = init if h == 0 else 0
        for k in range(16):
            w = 16 * h + k
            u = words[w]
            x = c ^ u
            if je[h] is not None and (je[h] >> 2) == w:
                t = je[h] & 3
                ax = c >> (8 * t)
                for i in range(t):
                    ax ^= TAB[t - 1 - i][(x >> (8 * i)) & 0xFF]
                cap[h] = ax
            if js[h] is not None and (js[h] >> 2) == w:
                t = js[h] & 3
                mlo = (1 << (8 * t)) - 1
                c = F(~(u | mlo) & 0xFFFFFFFF) ^ mlo
                continue
            c = F(x)
        R[h] = c
    tail = R[1] if js[1] is not None else (mul(R[0], X512) ^ R[1])
    return R[0], R[1], cap[0], cap[1], tail


def simulate_wave(buf, a0, offs, lens, r_lo, r_hi, out):
    """The records [r_lo, r_hi) (owned by one wave), from the tile holding
    r_lo's start to the tile holding r_hi-1's end event."""
    t_first = (offs[r_lo] - a0) >> 13
    t_last = (offs[r_hi - 1] + lens[r_hi - 1] - a0) >> 13
    carry = 0
    bt = r_lo
    for t in range(t_first, t_last + 1):
        T0 = a0 + 8192 * t
        TE = T0 + 8192
        cnt = 0
        while bt + cnt < r_hi and offs[bt + cnt] + lens[bt + cnt] < TE:
            cnt += 1
        ends = [[] for _ in range(64)]
        starts = [[] for _ in range(64)]
        for i in range(cnt + 1):
            r = bt + i
            if r >= r_hi or lens[r] < 64:
                continue
            if i < cnt:
                e = offs[r] + lens[r] - T0
                ends[e >> 7].append(e & 127)
            s = offs[r] - T0
            if 0 <= s < 8192:
                starts[s >> 7].append(s & 127)
        L = []
        for l in range(64):
            o = T0 + 128 * l
            ws = [int.from_bytes(buf[o + 4 * i:o + 4 * i + 4], "little") for i in range(32)]
            L.append(chunk_lane(ws, ends[l], starts[l], carry if l == 0 else 0))
        G = []
        for l in range(64):
            nxt = next((c for c in range(l + 1, 64) if ends[c]), 64)
            G.append(mul(L[l][4], xpow(1024 * (nxt - 1 - l))))
        X, acc = [], 0
        for g in G:
            acc ^= g
            X.append(acc)
        Y = lambda c: X[c - 1] if c >= 1 else 0  # noqa: E731
        for i in range(cnt):
            r = bt + i
            if lens[r] < 64:  # the window lane's direct checksum
                out[r] = zlib.crc32(buf[offs[r]:offs[r] + lens[r]])
                continue
            e = offs[r] + lens[r] - T0
            c, j = e >> 7, e & 127
            s = offs[r] - T0
            H = Y(c) ^ (Y(s >> 7) if s >= 0 else 0)
            h = 1 if j >= 64 else 0
            R0, R1, cap0, cap1, _ = L[c]
            P = mul(H, X512) ^ R0 if h else H
            v = mul(P, xpow(8 * (j - 64 * h))) ^ (cap1 if h else cap0)
            out[r] = (~v) & 0xFFFFFFFF
        ls = max((l for l in range(64) if starts[l]), default=None)
        carry = X[63] ^ (Y(ls) if ls is not None else 0)
        bt += cnt
    assert bt == r_hi


def simulate(data, offs, lens, waves=3):
    """data: the buffer the offsets index; the records sorted and not
    overlapping.  The records are cut into `waves` byte-balanced ranges."""
    n = len(offs)
    dend = offs[-1] + lens[-1]
    a0 = offs[0] & ~127
    buf = bytes(data) + bytes(2 * 8192 + 128)
    out = [None] * n
    cuts = [0]
    for w in range(1, waves):
        target = offs[0] + (dend - offs[0]) * w // waves
        cuts.append(next((r for r in range(n) if offs[r] >= target), n))
    cuts.append(n)
    for w in range(waves):
        if cuts[w] < cuts[w + 1]:
            simulate_wave(buf, a0, offs, lens, cuts[w], cuts[w + 1], out)
    return out


def gen(rnd, nrec, kind):
    """Record lengths and gaps of a test batch."""
    if kind == "packed64":
        lens, gaps = [64] * nrec, [0] * nrec
    elif kind == "wal":  # WAL payloads: Insert (13-byte header) / Remove (9-byte header)
        lens = [rnd.choice([0, 1, 5, 17, 40, 63, 64, 65, 100, 128, 300, 1000, 5000, 9000]) for _ in range(nrec)]
        gaps = [rnd.choice([13, 9]) for _ in range(nrec)]
    elif kind == "tiny":
        lens = [rnd.randrange(0, 40) for _ in range(nrec)]
        gaps = [rnd.choice([13, 9]) for _ in range(nrec)]
    else:
        lens = [rnd.choice([64, 65, 67, 100, 127, 128, 129, 191, 192, 255, 256, 300, 1000, 5000, 9000])
                for _ in range(nrec)]
        gaps = [rnd.choice([0, 0, 1, 3, 4, 13, 64]) for _ in range(nrec)]
    lead = rnd.randrange(0, 128)
    offs, p = [], lead
    for ln, g in zip(lens, gaps):
        p += g
        offs.append(p)
        p += ln
    return offs, lens, p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    rnd = random.Random(a.seed)
    fails = 0
    for kind in ("packed64", "mixed", "wal", "tiny"):
        offs, lens, end = gen(rnd, a.records, kind)
        data = bytes(rnd.randrange(256) for _ in range(end + 64))
        got = simulate(data, offs, lens)
        want = [zlib.crc32(data[s:s + ln]) for s, ln in zip(offs, lens)]
        bad = sum(1 for x, y in zip(got, want) if x != y)
        print(f"{kind}: {len(lens)} records, {bad} mismatches")
        fails += bad
    raise SystemExit(1 if fails else 0)


if __name__ == "__main__":
    main()
