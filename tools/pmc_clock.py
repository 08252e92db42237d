"""Per-dispatch effective clock from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass:
GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / the dispatch's duration
(MI355X_MICROARCH.md, "DVFS give-back"), for the dispatches whose kernel name
contains PATTERN, in dispatch order.

  python3 tools/pmc_clock.py <pmc output dir> [PATTERN]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "crc32_stream_kernel"
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if pat not in r["Kernel_Name"] or r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                    continue
                k = int(r["Dispatch_Id"])
                e = rows.setdefault(k, [int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0.0, r["Kernel_Name"]])
                e[2] += float(r["Counter_Value"])
    print(f"{'dispatch':>9} {'ms':>8} {'cycles (M)':>11} {'GHz':>6}  kernel")
    for k in sorted(rows):
        s, e, gui, name = rows[k]
        ns = e - s
        print(f"{k:9d} {ns / 1e6:8.3f} {gui / 8 / 1e6:11.2f} {gui / 8 / ns:6.3f}  {name.split('(')[0][:50]}")


if __name__ == "__main__":
    main()
