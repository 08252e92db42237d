#!/usr/bin/env python3
"""Merge pmc_summary.py outputs into profiles/pmc_traffic.json (the bench's
roofline.traffic source): python3 tools/pmc_merge.py ROUND summary.json ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rnd = sys.argv[1]
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(p)) if os.path.exists(p) else {}
    for f in sys.argv[2:]:
        for k, v in json.load(open(f)).items():
            v["round"] = rnd
            d[k] = v
    with open(p, "w") as fh:
        json.dump(d, fh, indent=1)


if __name__ == "__main__":
    main()
