#!/usr/bin/env python3
"""Kernel-trace statistics from a rocprofv3 rocpd database (results.db) or
kernel_trace.csv: per kernel name, calls / total / average / median / min / max (us)."""
import csv
import glob
import os
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        for name, dur in con.execute("select name, duration from kernels"):
            yield name, float(dur)
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                yield r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"])


def main():
    for arg in sys.argv[1:]:
        files = [arg] if os.path.isfile(arg) else (glob.glob(os.path.join(arg, "**", "*.db"), recursive=True) +
                                                   glob.glob(os.path.join(arg, "**", "*kernel_trace.csv"), recursive=True))
        agg = {}
        for f in files:
            for n, d in rows(f):
                agg.setdefault(n.split("(")[0][:90], []).append(d / 1000.0)
        print(f"== {arg}")
        print(f"{'kernel':92s} {'calls':>5s} {'total_us':>12s} {'avg_us':>10s} {'median_us':>10s} {'min_us':>10s} "
              f"{'max_us':>10s}")
        for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            med = sorted(v)[len(v) // 2] if len(v) % 2 else sum(sorted(v)[len(v) // 2 - 1:len(v) // 2 + 1]) / 2
            print(f"{n:92s} {len(v):5d} {sum(v):12.1f} {sum(v) / len(v):10.1f} {med:10.1f} {min(v):10.1f} {max(v):10.1f}")


if __name__ == "__main__":
    main()
