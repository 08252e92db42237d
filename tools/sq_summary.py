#!/usr/bin/env python3
"""Per-dispatch counters of one kernel from a rocprofv3 --pmc --kernel-trace
csv directory: each counter summed over its instances (XCDs / SEs), the
dispatch time, and the effective clock GRBM_GUI_ACTIVE / 8 / time
(MI355X_MICROARCH.md, "DVFS give-back"); then the mean over all but the first
dispatch.
  python3 tools/sq_summary.py <pmc output dir> [PATTERN]"""
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
                if pat not in r["Kernel_Name"]:
                    continue
                k = int(r["Dispatch_Id"])
                e = rows.setdefault(k, {"_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                        "_name": r["Kernel_Name"].split("(")[0]})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not rows:
        print("no dispatch of", pat)
        return
    names = sorted({c for e in rows.values() for c in e if not c.startswith("_")})
    for k in sorted(rows):
        e = rows[k]
        ghz = e.get("GRBM_GUI_ACTIVE", 0.0) / 8 / e["_ns"]
        print(f"dispatch {k} {e['_name']}: {e['_ns'] / 1e6:.3f} ms, {ghz:.3f} GHz, " +
              ", ".join(f"{c} {e.get(c, 0):.4g}" for c in names))
    # per kernel (template instance): the mean over its dispatches but the first
    for kname in sorted({e["_name"] for e in rows.values()}):
        ks = [k for k in sorted(rows) if rows[k]["_name"] == kname]
        keep = [rows[k] for k in ks[1:]] or [rows[k] for k in ks]
        ms = sum(e["_ns"] for e in keep) / len(keep) / 1e6
        print(f"{kname}: mean of {len(keep)}: {ms:.3f} ms")
        for c in names:
            v = sum(e.get(c, 0.0) for e in keep) / len(keep)
            extra = f"  ({v / 8 / (ms * 1e6):.3f} GHz, {v / 8 / 1e6:.2f} M cycles)" if c == "GRBM_GUI_ACTIVE" else ""
            print(f"  {c:24s} {v:.4g}{extra}")


if __name__ == "__main__":
    main()
