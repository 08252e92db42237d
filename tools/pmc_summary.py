#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per
launch of the dominant kernel.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE counts 128-B read requests as 64 B -> x2 for wide streaming reads;
WRITE_SIZE is exact for 16-B-per-lane stores.  Both are in KiB."""
import csv
import glob
import json
import os
import re
import sys


def per_kernel(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    rows.append((r.get("Kernel_Name", ""), float(r["Counter_Value"])))
    out = {}
    for k, v in rows:
        out.setdefault(k, []).append(v)
    return out


def main():
    fd, wd, workload = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = per_kernel(fd, "FETCH_SIZE")
    write = per_kernel(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if not any(n in k for n in ("crc32_fixed_kernel", "crc32_wring_kernel", "crc32_desc_kernel", "crc32_walk_kernel",
                                    "crc32_stream_kernel", "sha256_kernel")):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2 * 1024 * sum(f) / len(f) if f else None
        wb = 1024 * sum(w) / len(w) if w else None
        res[k] = {"dispatches": max(len(f), len(w)), "fetch_bytes_corrected": fb, "write_bytes": wb,
                  "hbm_bytes_per_launch": (fb or 0) + (wb or 0)}
    # the dominant kernel among the non-diagnostic ones (crc_ablate variants
    # carry a nonzero ABLATE template argument)
    def diagnostic(k):
        m = re.search(r"crc32_(stream|wring|walk)_kernel<(\d+), (\d+)", k)
        if not m:
            return False
        return int(m.group(2) if m.group(1) == "stream" else m.group(3)) != 0
    real = {k: v for k, v in res.items() if not diagnostic(k)} or res
    dom = max(real.values(), key=lambda x: x["hbm_bytes_per_launch"]) if real else None
    print(json.dumps({workload: {"hbm_bytes_per_launch": dom["hbm_bytes_per_launch"] if dom else None,
                                 "kernels": res,
                                 "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes; "
                                           "FETCH_SIZE x2 (gfx950 128-B requests tallied as 64 B)"}}, indent=1))


if __name__ == "__main__":
    main()
