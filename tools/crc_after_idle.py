#!/usr/bin/env python3
"""Does the stream kernel start slow after the GPU idles or runs
latency-bound work?  (Inside the WAL replay the CRC pass follows ~4 ms of
the header walk and runs ~0.8 ms longer than the same pass back to back,
profiles/r06/final2.)  Config 3's batch (bench.py's records and bytes), the
CRC pass timed with HIP events on its stream after each kind of prelude:

  back-to-back   the previous pass
  host-idle      a 4 ms host sleep after a synchronize
  gpu-spin       a 4 ms spin kernel on the stream (torch.cuda._sleep)
  hbm-copy       a 4 GiB device copy on the stream (HBM busy right before)
  mfma-4ms       ~4 ms of bf16 matmuls on the stream (power-hungry right before)

  python3 tools/crc_after_idle.py [--rounds 4]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--idle-ms", type=float, default=4.0)
    ap.add_argument("--sweep", default="", help="comma list of host-idle ms: the pass after each (instead of the preludes)")
    ap.add_argument("--mfma-sweep", default="",
                    help="comma list of ms of bf16 matmuls run after an --idle-ms host idle, right before the pass")
    a = ap.parse_args()
    import torch
    import bench
    from lsm_storage_engine_amd.device import Context, gen_zipf_lengths
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    sptr = stream.cuda_stream
    ctx = Context(0)
    nrec = 1 << 26
    offs, lens, nbytes, byte_off = bench.config3_shard(gen_zipf_lengths, bench.SEED[3], nrec, 0)
    data = ctx.alloc(nbytes + 64)
    ctx.gen_stream(data.ptr, bench.SEED[3], byte_off, nbytes, sptr)
    out = ctx.alloc(4 * nrec)
    d_off, d_len = ctx.alloc(8 * nrec), ctx.alloc(4 * nrec)
    d_off.upload(offs)
    d_len.upload(lens)
    ctx.sync(sptr)
    src = torch.empty(1 << 30, dtype=torch.int32, device="cuda")  # 4 GiB
    dst = torch.empty_like(src)
    # the spin kernel's rate: cycles per ms
    with torch.cuda.stream(stream):
        torch.cuda._sleep(1_000_000)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record(stream)
        torch.cuda._sleep(10_000_000)
        e1.record(stream)
    torch.cuda.synchronize()
    cyc_per_ms = 10_000_000 / e0.elapsed_time(e1)

    def crc():
        ctx.crc32_device(data.ptr, d_off.ptr, d_len.ptr, nrec, out.ptr, sptr)

    def timed_crc():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        crc()
        e.record(stream)
        return s, e

    res = {k: [] for k in ("back-to-back", "host-idle", "gpu-spin", "hbm-copy", "mfma-4ms")}
    ma = torch.randn(8192, 8192, dtype=torch.bfloat16, device="cuda")
    mb = torch.randn(8192, 8192, dtype=torch.bfloat16, device="cuda")
    mc = torch.empty(8192, 8192, dtype=torch.bfloat16, device="cuda")
    with torch.cuda.stream(stream):  # the matmul's time: iterations for ~idle_ms
        torch.matmul(ma, mb, out=mc)
        e0.record(stream)
        for _ in range(4):
            torch.matmul(ma, mb, out=mc)
        e1.record(stream)
    torch.cuda.synchronize()
    mm_iters = max(1, int(round(a.idle_ms / (e0.elapsed_time(e1) / 4))))
    crc()
    ctx.sync(sptr)
    if a.mfma_sweep:  # idle, then X ms of matmuls, then the pass (X = 0: idle alone)
        per = (e0.elapsed_time(e1) / 4)
        xs = [float(x) for x in a.mfma_sweep.split(",")]
        sw = {x: [] for x in xs}
        for _ in range(a.rounds):
            for x in xs:
                crc()
                ctx.sync(sptr)
                time.sleep(a.idle_ms / 1e3)
                with torch.cuda.stream(stream):
                    for _ in range(int(round(x / per))):
                        torch.matmul(ma, mb, out=mc)
                s, e = timed_crc()
                torch.cuda.synchronize()
                sw[x].append(s.elapsed_time(e))
        print(json.dumps({"what": f"config-3 pass (ms) after a {a.idle_ms} ms idle and X ms of bf16 matmuls",
                          "matmul_ms": round(per, 3),
                          "ms": {str(k): [round(v, 3) for v in vs] for k, vs in sw.items()},
                          "median_ms": {str(k): round(sorted(vs)[len(vs) // 2], 3) for k, vs in sw.items()}}))
        return
    if a.sweep:  # the pass after host idles of several lengths, interleaved
        idles = [float(x) for x in a.sweep.split(",")]
        sw = {x: [] for x in idles}
        for _ in range(a.rounds):
            for x in idles:
                crc()
                crc()
                ctx.sync(sptr)
                time.sleep(x / 1e3)
                s, e = timed_crc()
                torch.cuda.synchronize()
                sw[x].append(s.elapsed_time(e))
        print(json.dumps({"what": "config-3 stream-kernel pass (ms, HIP events) after a host idle of each length",
                          "ms": {str(k): [round(v, 3) for v in vs] for k, vs in sw.items()},
                          "median_ms": {str(k): round(sorted(vs)[len(vs) // 2], 3) for k, vs in sw.items()}}))
        return
    for _ in range(a.rounds):
        # back-to-back: the second of two passes
        crc()
        s, e = timed_crc()
        torch.cuda.synchronize()
        res["back-to-back"].append(s.elapsed_time(e))
        ctx.sync(sptr)
        time.sleep(a.idle_ms / 1e3)
        s, e = timed_crc()
        torch.cuda.synchronize()
        res["host-idle"].append(s.elapsed_time(e))
        with torch.cuda.stream(stream):
            torch.cuda._sleep(int(cyc_per_ms * a.idle_ms))
        s, e = timed_crc()
        torch.cuda.synchronize()
        res["gpu-spin"].append(s.elapsed_time(e))
        with torch.cuda.stream(stream):
            dst.copy_(src)
        s, e = timed_crc()
        torch.cuda.synchronize()
        res["hbm-copy"].append(s.elapsed_time(e))
        with torch.cuda.stream(stream):  # a power-hungry prelude: bf16 matmuls on the MFMA units
            for _ in range(mm_iters):
                torch.matmul(ma, mb, out=mc)
        s, e = timed_crc()
        torch.cuda.synchronize()
        res["mfma-4ms"].append(s.elapsed_time(e))
    print(json.dumps({"what": "config-3 stream-kernel pass (ms, HIP events) after each prelude",
                      "idle_ms": a.idle_ms, "spin_cycles_per_ms": round(cyc_per_ms),
                      "ms": {k: [round(x, 3) for x in v] for k, v in res.items()},
                      "median_ms": {k: round(sorted(v)[len(v) // 2], 3) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
