#!/usr/bin/env python3
"""Instruction mix of a kernel's largest loop in a hipcc --save-temps .s file.

  python3 tools/isa_loop.py file.s kernel_symbol [...]
"""
import collections
import re
import sys


def body(s, name):
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    return s[i:j]


def loop_mix(b):
    lines = b.split("\n")
    labels = {l.split(":")[0]: k for k, l in enumerate(lines) if re.match(r"^\.LBB\d+_\d+:", l)}
    best = None
    for k, l in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < k:
                size = k - labels[t]
                if best is None or size > best[0]:
                    best = (size, labels[t], k)
    _, a, z = best
    loop = [x.strip() for x in lines[a:z + 1] if x.strip() and not x.strip().startswith((";", "."))]
    cnt = collections.Counter()
    for x in loop:
        op = x.split()[0]
        if op.startswith("v_"):
            cnt["valu"] += 1
        elif op.startswith("ds_"):
            cnt["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            cnt["vmem"] += 1
        elif op.startswith("s_waitcnt"):
            cnt["waitcnt"] += 1
        elif op.startswith("s_"):
            cnt["salu"] += 1
    ops = collections.Counter(x.split()[0] for x in loop if x.split()[0].startswith("v_"))
    return len(loop), dict(cnt), ops


def main():
    s = open(sys.argv[1]).read()
    for name in sys.argv[2:]:
        n, cnt, ops = loop_mix(body(s, name))
        print(name, "loop instructions", n, cnt)
        print("  top VALU:", ops.most_common(24))


if __name__ == "__main__":
    main()
