#!/usr/bin/env python3
"""Bytes the L2 requested from the fabric, by request size, per launch of each
kernel: 128 * TCC_EA0_RDREQ_128B + 64 * TCC_EA0_RDREQ_64B + 32 *
TCC_EA0_RDREQ_32B, and the share of the requests that went to DRAM
(TCC_EA0_RDREQ_DRAM), from rocprofv3 --pmc passes (the request counts that
FETCH_SIZE's fixed x2 correction assumes; MI355X_MICROARCH.md: "other access
widths are uncalibrated").

  python3 tools/pmc_reqsize.py <pass dir> [<pass dir> ...]
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import per_kernel  # noqa: E402

NAMES = ["TCC_EA0_RDREQ_sum", "TCC_BUBBLE_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_32B_sum",
         "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_RDREQ_DRAM_32B_sum"]


def main():
    got = {}
    for d in sys.argv[1:]:
        for c in NAMES:
            for k, v in per_kernel(d, c).items():
                got.setdefault(k, {})[c] = sum(v) / len(v)  # per dispatch
    out = {}
    for k, c in got.items():
        if max(c.values(), default=0) < 1e6:
            continue
        b = (128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0)
             + 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0))
        out[k] = {**{n: c.get(n) for n in NAMES}, "read_bytes_by_size": b,
                  "fetch_size_x2_equiv": 128 * c.get("TCC_EA0_RDREQ_sum", 0),
                  # requests to DRAM (the rest of RDREQ are served by the Infinity Cache / other agents)
                  "dram_request_fraction": c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / max(1.0, c.get("TCC_EA0_RDREQ_sum", 0))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
