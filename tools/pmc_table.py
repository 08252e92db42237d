#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter passes (one or more output
directories): kernel -> counter -> mean over dispatches (summed over the
counter's instances, as rocprofv3 reports them)."""
import csv
import glob
import os
import sys


def main():
    acc = {}
    for d in sys.argv[1:]:
        tag = os.path.basename(d.rstrip("/"))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r.get("Kernel_Name", "")
                    if "crc32" not in k and "scan_phase" not in k and "sha256" not in k:
                        continue
                    short = k.split("(")[0].replace("void lsmck::", "")[:60]
                    key = (tag.rsplit("_g", 1)[0], short)
                    acc.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for (tag, k), cs in sorted(acc.items()):
        print(f"[{tag}] {k}")
        for c, v in sorted(cs.items()):
            print(f"    {c:40s} {sum(v) / len(v):16.4g}   (n={len(v)})")


if __name__ == "__main__":
    main()
