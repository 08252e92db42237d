#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing (gfx950).

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude -Ilsm_storage_engine_amd/csrc \\
        --cuda-device-only -S lsm_storage_engine_amd/csrc/lsmck_crc32.hip -o /tmp/crc.s
  python3 tools/isa_stats.py /tmp/crc.s crc32_stream_kernelILi0E [--blocks]

Counts by class (VALU, SALU, LDS, vector memory, waits, branches) for the
whole kernel, and with --blocks per basic block (label, size, LDS ops,
lgkmcnt waits), to see where a loop body waits on LDS / scalar loads.
"""
import re
import sys
from collections import Counter


def kind(op):
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("v_mfma",)):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return op


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", s, re.M)
    if not m:
        sys.exit(f"no kernel matching {pat}")
    i = m.start()
    j = s.index(".Lfunc_end", i)
    lines = s[i:j].splitlines()
    total = Counter()
    blocks = []
    cur = ["<entry>", Counter(), 0]
    for ln in lines:
        if re.match(r"^\.LBB\S*:", ln) or re.match(r"^_Z\S*:", ln):
            blocks.append(cur)
            cur = [ln.split(":")[0], Counter(), 0]
            continue
        t = ln.strip()
        if not ln.startswith("\t") or not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        k = kind(op)
        total[k] += 1
        cur[1][k] += 1
        cur[2] += 1
        if op == "s_waitcnt" and "lgkmcnt(0)" in t:
            cur[1]["lgkm0"] += 1
            total["lgkm0"] += 1
        if op == "s_waitcnt" and "vmcnt(0)" in t:
            cur[1]["vm0"] += 1
            total["vm0"] += 1
    blocks.append(cur)
    print(m.group(1), sum(v for k, v in total.items() if k not in ("lgkm0", "vm0")), dict(total))
    if "--blocks" in sys.argv:
        for name, c, n in blocks:
            if n:
                print(f"  {name:14s} {n:5d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
