#!/usr/bin/env python3
"""Host simulation of crc32_walk_kernel's record map (lsmck_crc32.hip), lane
by lane, on index arithmetic only: superblock cuts, the three-window ring,
the start-bit mask, the per-lane (record, segment) map, the cursor and the
Horner emission order.  It checks that every valid lane maps to the segment a
plain enumeration gives, that every record is emitted exactly once, at the
lane holding its last segment's run head, and that no valid lane reads
outside its record.  Used before running a changed kernel on the GPU.

  python3 tools/walk_sim.py [trials]
"""
import sys

import numpy as np

SB = 256


def nseg(l):
    return np.where(l == 0, 1, (l.astype(np.int64) + 127) // 128)


def simulate(lens, nw):
    n = len(lens)
    ns = nseg(lens)
    nsb = (n + SB - 1) // SB
    sb_sum = np.array([ns[b * SB:(b + 1) * SB].sum() for b in range(nsb)], dtype=np.int64)
    pre = np.concatenate([[0], np.cumsum(sb_sum)[:-1]]).astype(np.int64)
    S = int(sb_sum.sum())
    seg_rec = np.repeat(np.arange(n), ns)           # reference: record of every segment
    seg_q = np.concatenate([np.arange(k) for k in ns]) if n else np.zeros(0, np.int64)
    emitted = np.zeros(n, dtype=np.int64)
    lanes = np.arange(64)

    def cut(w):
        if w >= nw:
            return nsb
        target = (S // nw) * w + (S % nw) * w // nw
        return int(np.searchsorted(pre, target, side="left"))

    for wave in range(nw):
        b0, b1 = cut(wave), cut(wave + 1)
        if b0 >= b1:
            continue
        r0, r1 = b0 * SB, min(n, b1 * SB)
        segs = (pre[b1] if b1 < nsb else S) - pre[b0]
        ntile = (segs + 63) // 64
        run_seg0 = int(pre[b0])                      # global segment of the run's first segment

        def win(w0):
            r = w0 + lanes
            ok = r < r1
            rr = np.where(ok, r, r1 - 1)
            ln = lens[rr]
            nsg = np.where(ok, nseg(ln), 0)
            inc = np.cumsum(nsg)
            return {"len": ln, "ok": ok, "p": inc - nsg, "tot": int(inc[-1]), "r": rr}

        cur, nxt, prew = win(r0), win(r0 + 64), win(r0 + 128)
        wc0, Bc = r0, 0
        Bn = Bc + cur["tot"]
        G, rg, qg = 0, r0, 0
        for t in range(ntile):
            def bits(W, rel):
                s = rel + W["p"]
                m = W["ok"] & (s >= 1) & (s <= 63)
                return set(s[m].tolist())
            starts = bits(cur, Bc - G) | bits(nxt, Bn - G)
            rec = np.zeros(64, np.int64)
            q = np.zeros(64, np.int64)
            for l in range(64):
                below = [x for x in starts if 1 <= x <= l]
                rec[l] = rg + len(below)
                q[l] = l - max(below) if below else qg + l
            valid = G + lanes < segs
            idx = np.where(valid, rec - wc0, 0)
            assert (idx[valid] >= 0).all() and (idx[valid] < 128).all(), ("window", wave, t)
            ln = np.where(idx < 64, cur["len"][idx & 63], nxt["len"][idx & 63])
            # the lane's record and segment agree with the enumeration
            gseg = run_seg0 + G + lanes
            for l in np.nonzero(valid)[0]:
                assert rec[l] == seg_rec[gseg[l]] and q[l] == seg_q[gseg[l]], ("map", wave, t, l)
                assert ln[l] == lens[rec[l]]
            k = np.where(valid, nseg(ln) - 1 - q, 0)
            assert (k[valid] >= 0).all()
            first = valid & (q == 0)
            head = valid & ((lanes == 0) | first)
            ends = head & (lanes + k <= 63)
            for l in np.nonzero(ends)[0]:
                emitted[rec[l]] += 1
            # cursor
            k63 = int(k[63]) if valid[63] else 0
            rg = int(rec[63]) + (0 if k63 else 1)
            qg = int(q[63]) + 1 if k63 else 0
            G += 64
            rot = rg >= wc0 + 64
            if rot:
                cur = nxt
                nxt = prew
                wc0 += 64
                Bc, Bn = Bn, Bn + cur["tot"]
            prew = win(wc0 + 128)
    assert (emitted == 1).all(), np.nonzero(emitted != 1)[0][:10]
    return S


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    rng = np.random.default_rng(1)
    for tr in range(trials):
        n = int(rng.integers(1, 3000))
        kind = tr % 5
        if kind == 0:
            lens = rng.integers(0, 700, n)
        elif kind == 1:
            lens = rng.integers(0, 130, n)
        elif kind == 2:
            lens = rng.integers(0, 300, n)
            lens[rng.integers(0, n, 3)] = rng.integers(1 << 16, 1 << 20, 3)
        elif kind == 3:
            lens = np.full(n, 4096)
        else:
            lens = np.zeros(n, dtype=np.int64)
        nw = int(rng.choice([1, 3, 7, 64]))
        simulate(np.asarray(lens, dtype=np.int64), nw)
    print("walk map simulation ok:", trials, "trials")


if __name__ == "__main__":
    main()
