"""Timeline of the last kernels in a rocprofv3 kernel trace: start and end
(ms, relative to the first kernel shown), queue, grid and name -- to see
which kernels ran beside which (the pipelined WAL replay's walk beside its
CRC passes).

  python3 tools/kt_timeline.py <dir with *kernel_trace.csv> [--last N] [--after NAME]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=60)
    ap.add_argument("--after", default="", help="start at the last kernel whose name contains this")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Grid_Size_X"],
                             r["Kernel_Name"]))
    rows.sort()
    if a.after:
        idx = [i for i, r in enumerate(rows) if a.after in r[4]]
        if idx:
            rows = rows[idx[-1]:]
    rows = rows[-a.last:]
    t0 = rows[0][0]
    for s, e, q, g, name in rows:
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} q{q:>3} grid {g:>9} {name[:90]}")


if __name__ == "__main__":
    main()
