#!/usr/bin/env python3
"""Where the host side of a host-resident batch runs on a multi-socket node
(pinned staging NUMA-local to the GPU's PCIe root).

Prints the device's NUMA node and the host's node count, then for each
"stage_numa" setting (-2 auto = the device's node, -1 = HIP's default
placement and free-floating copy threads, and every node forced) in a fresh
context:
  * which node the pages of a pinned buffer from lsmck_host_alloc_pinned
    landed on (move_pages), and
  * the rate of a 8 GiB pageable host CRC batch of 4 KiB blocks (copy into the
    pinned staging slots on the context's threads, then DMA; the GPU's CRCs
    checked against the first batch's), best of 3,
  * the rate of the same batch from a pinned buffer of that context (DMA only).
One JSON line.  python3 tools/numa_probe.py [--gib 8]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lsm_storage_engine_amd.device import Context  # noqa: E402

SYS_MOVE_PAGES = 279  # x86_64


def page_nodes(ptr, nbytes, samples=64):
    """NUMA node of `samples` pages spread over [ptr, ptr+nbytes) (move_pages, query only)."""
    libc = C.CDLL(None, use_errno=True)
    page = os.sysconf("SC_PAGE_SIZE")
    n = max(1, min(samples, nbytes // page))
    addrs = (C.c_void_p * n)(*[ptr + (i * (nbytes // n) // page) * page for i in range(n)])
    status = (C.c_int * n)()
    libc.syscall.restype = C.c_long
    rc = libc.syscall(C.c_long(SYS_MOVE_PAGES), C.c_int(0), C.c_ulong(n), addrs, None, status, C.c_int(0))
    if rc != 0:
        return {"error": os.strerror(C.get_errno())}
    out = {}
    for s in status:
        out[str(s)] = out.get(str(s), 0) + 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    a = ap.parse_args()
    nodes = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit()])
    n = int(a.gib * (1 << 30)) // 4096
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, size=n * 4096, dtype=np.uint8)  # pageable source, touched by this thread
    probe = Context(0)
    dev_node = probe.get_stat("numa_node")
    probe.close()
    modes = [-2, -1] + list(range(nodes))
    out = {"nodes": nodes, "device_node": dev_node, "bytes": n * 4096, "modes": {}}
    want = None
    for m in modes:
        ctx = Context(0)
        ctx.set_option("stage_numa", m)
        pb = ctx.alloc_pinned(256 << 20)
        pb.array[:] = 1  # (touch: pages are pinned at allocation already)
        where = page_nodes(pb.ptr, pb.nbytes)
        pb.free()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            crc = ctx.crc32_fixed(data, 4096, 4096, n)
            ts.append(time.perf_counter() - t)
        if want is None:
            want = crc
        ok = bool(np.array_equal(crc, want))
        src = ctx.alloc_pinned(n * 4096)
        src.array[:] = data
        tp = []
        for _ in range(3):
            t = time.perf_counter()
            crc2 = ctx.crc32_fixed(src.array, 4096, 4096, n, pinned=True)
            tp.append(time.perf_counter() - t)
        ok = ok and bool(np.array_equal(crc2, want))
        src_where = page_nodes(src.ptr, src.nbytes)
        src.free()
        out["modes"][str(m)] = {"stage_numa_node": ctx.get_stat("stage_numa_node"), "pinned_pages_on_node": where,
                                "pageable_GiBps": round(n * 4096 / min(ts) / (1 << 30), 2),
                                "pinned_src_GiBps": round(n * 4096 / min(tp) / (1 << 30), 2),
                                "pinned_src_pages_on_node": src_where, "crcs_match": ok}
        print(f"stage_numa {m}: {out['modes'][str(m)]}", file=sys.stderr, flush=True)
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
