#!/usr/bin/env python3
"""Benchmark of the MI355X checksum path (BASELINE.json metric:
"GiB/s device-resident batched record checksum; % of HBM3E read BW").

One step = one pass of the hot path (lsmck_crc32_batch*) over one batch of
synthetic records already resident in HBM.  Default workload at every N is
BASELINE config 3, the north_star's "synthetic variable-length KV records
(64 B-64 KiB) at 1, 2, 4 and 8 MI355X": 2^26 Zipf-length records per GPU
packed back to back (~97 GiB, the largest single-GPU config).  With --gpus N
there is one process per GPU and rank r checksums records [r*2^26, (r+1)*2^26)
of ONE global config-3 stream (its lengths from the counter-based generator
at record r*2^26, its bytes at the stream offset where rank r-1's end) --
weak scaling, record-sharded, no data-path collective; the control plane
(barrier, max of per-rank times, per-rank summary digests against the
oracle's, tests/golden/summaries.json config3_shards) goes over
torch.distributed (gloo).  Rank 0's shard is the N = 1 workload itself, so
the 1 -> N curve is like for like.  Every line also carries BASELINE config 4
as "config4": the fixed 4 KiB block shard (2^26 blocks = 256 GiB per GPU,
shard r = blocks [r*2^26, (r+1)*2^26) of config 2's stream), timed the same
way after the config-3 buffers are freed.  --config 2 / 1 run the fixed 4 KiB
blocks (64 GiB; config 4's shard at N > 1) / the 256 B WAL payloads.

`python bench.py --gpus N` outside torch.distributed.run starts
`torch.distributed.run --nproc-per-node N` on itself as a child process
(before anything touches the GPU) and exits with its status; under a launcher
WORLD_SIZE must equal --gpus.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3|2|1]
                  [--blocks-per-gpu B] [--no-cpu-baseline]

Prints ONE JSON line on rank 0 (see DESIGN.md section 5 for every field).
"""
import argparse
import json
import re
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# torch and liblsmck are imported in main(), after relaunch(): nothing may
# touch the GPU in a process that then starts the N-rank launcher

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, GB/s (MI355X_MICROARCH.md chip table)
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12  # full-rate VALU issue slots/s: 256 CU x 128 lanes/clk x 2.4 GHz
# VALU issue slots per SHA-256 compression in sha256_kernel's main loop (gfx950
# ISA, per block: 576 v_alignbit_b32 + 241 v_add3_u32 + 16 v_perm_b32, which
# issue at half rate (tools/microbench_valu.hip: 62 vs 103-110 lane-ops/clk/CU
# for v_add_u32 / v_xor_b32 / v_bitop3_b32), + 572 full-rate (352 v_bitop3,
# 118 v_add, 96 v_lshrrev, 6 other): 833*2 + 572 = 2,238.  r01 v6: Ch and Maj
# are one v_bitop3 each, and the funnel + byte swap one v_perm (the earlier
# kernel issued 1,553 instructions per block).
SHA_OPS_PER_BLOCK = 2238
METRIC = "GiB/s device-resident batched record checksum; % of HBM3E read BW"
CONFIG3_SHARDS = {1 << 26: "config3_shards", 1 << 20: "config3_shards_small"}  # records per rank -> golden key
SEED = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=0, choices=[0, 1, 2, 3],
                    help="0 (default): config 3 (records [r*2^26, (r+1)*2^26) of one global stream per rank); "
                         "2: config 2's blocks (config 4's 2^26-block shard per rank at N > 1)")
    ap.add_argument("--no-config4", action="store_true",
                    help="skip the config-4 block-shard sub-measurement of the config-3 line")
    ap.add_argument("--c4-blocks", type=int, default=0,
                    help="blocks per rank of the config-4 sub-measurement (default 2^26; 2^26/N when the ranks "
                         "share one GPU)")
    ap.add_argument("--blocks-per-gpu", type=int, default=0, help="override the per-GPU record count")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-records", type=int, default=0)
    ap.add_argument("--variants", default="",
                    help="comma list of A/B variants timed in interleaved rounds, each a '+' list of "
                         "s<n> (crc_stream: 0 walking kernel only, 1 default), a<n> (crc_ablate: 3 payload "
                         "loads only, 2 stream kernel without loads), p<n> (sha_pair), b<n> (sha_bucket_shift), t<n> (sha_short_blocks), "
                         "f<n> (sha_bucket_from); '-' is the default")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-stream-ceiling", action="store_true",
                    help="skip the loads-only ceiling run of the same kernel (roofline.loads_only_ceiling)")
    ap.add_argument("--no-host-roundtrip", action="store_true",
                    help="skip the host-resident (pinned H2D + kernel + D2H) sample")
    ap.add_argument("--desc", action="store_true",
                    help="diagnostic: config 2's fixed blocks through the descriptor entry point")
    ap.add_argument("--digest", default="crc32", choices=["crc32", "sha256"],
                    help="crc32 = the WAL record checksum (headline); sha256 = the SSTable digest "
                         "(checksums.rs) over the same records, reported against its int32 VALU roof")
    ap.add_argument("--stream", type=int, default=1, choices=[0, 1],
                    help="descriptor batches: 1 = stream kernel (default), 0 = walking kernel (A/B)")
    ap.add_argument("--sorted", action="store_true",
                    help="descriptor batches with LSMCK_SORTED: the caller asserts its records are sorted inside "
                         "one readable span, so the device-side check of the descriptors is skipped")
    ap.add_argument("--wal-framed", action="store_true",
                    help="config 3's records framed as wal.rs Insert records (13-byte headers between the payloads)")
    ap.add_argument("--pack-align", type=int, default=1,
                    help="diagnostic: config 3 record offsets rounded up to this many bytes")
    return ap.parse_args()


def resolve_config(config, world):
    """--config 0 (default): BASELINE config 3 (north_star's variable-length
    records) at every N: rank r takes records [r*2^26, (r+1)*2^26) of one
    global stream."""
    return config or 3


def traffic_from_profiles(workload_key):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json),
    collected with rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes and
    corrected as MI355X_MICROARCH.md prescribes (FETCH_SIZE x 2 on gfx950)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(workload_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


# host cores for the all-cores CPU row: the GPU box gives a process 16 CPUs
CPU_ALL_CORES = int(os.environ.get("LSMCK_CPU_CORES", "16"))


def relaunch(a):
    """--gpus N outside a launcher: run N ranks under torch.distributed.run as a
    child process (one process per GPU) and return its exit status; under a
    launcher, WORLD_SIZE must match --gpus.  Returns None to run in-process."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus and not (a.gpus == 1 and int(ws) > 1 and "--gpus" not in sys.argv):
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {a.gpus}", file=sys.stderr)
            return 2
        return None
    if a.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as so:  # a free rendezvous port on the loopback
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def golden_summaries():
    p = os.path.join(ROOT, "tests", "golden", "summaries.json")
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def config3_shard(gen, seed, nrec, rank, gather=None, framed=False, align=1):
    """Rank r's share of one global config-3 stream: records [r*nrec,
    (r+1)*nrec) -- their lengths from the counter-based generator `gen` at
    record r*nrec -- laid out packed (or wal.rs-framed: a 13-byte header before
    every payload, wal.rs:178-182), and the stream byte offset of the shard's
    first byte: the sizes of the lower ranks' shards (gather: an all_gather of
    one value per rank; None at N = 1).  Returns (offs, lens, nbytes, byte_off)."""
    lens = gen(seed, nrec, first=rank * nrec)
    offs = np.zeros(nrec, dtype=np.uint64)
    if framed:
        offs[:] = 13  # payload i+1 starts len[i] + 13 after payload i
        offs[1:] += lens[:-1].astype(np.uint64)
        offs = np.cumsum(offs, dtype=np.uint64)
    else:
        slot = ((lens.astype(np.uint64) + (align - 1)) // align) * align  # align 1: packed back to back
        np.cumsum(slot[:-1], out=offs[1:])
    nbytes = int(offs[-1]) + int(lens[-1])
    byte_off = sum(gather(nbytes)[:rank]) if gather else 0
    return offs, lens, nbytes, byte_off


def config4_sub(a, ctx, stream, sptr, world, rank):
    """BASELINE config 4 on this rank: blocks [r*n4, (r+1)*n4) of config 2's
    4 KiB block stream (n4 = 2^26: 256 GiB per GPU), W warm-up steps, then K
    steps between barriers, the max wall time over ranks; per-rank digests
    against the oracle's (make_summaries.py config4) at full size."""
    share = bool(os.environ.get("LSMCK_BENCH_SHARE_GPU")) and world > 1
    n4 = a.c4_blocks or ((1 << 26) // world if share else (1 << 26))
    L = 4096
    d4, o4 = ctx.alloc(n4 * L + 64), ctx.alloc(4 * n4)
    ctx.gen_stream(d4.ptr, SEED[2], rank * n4 * L, n4 * L, sptr)

    def step4():
        ctx.crc32_fixed_device(d4.ptr, L, L, n4, o4.ptr, sptr)
    for _ in range(a.warmup):
        step4()
    ctx.sync(sptr)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        step4()
    e1.record(stream)
    ctx.sync(sptr)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    ev_ms = e0.elapsed_time(e1) / a.steps
    t = torch.tensor([wall], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t[0])
    import zlib
    mine = "%08x" % zlib.crc32(o4.download(np.uint8, count=4 * n4).tobytes())
    mine_t = {"rank": rank, "launch_ms_hip_events": round(ev_ms, 4), "summary_crc32": mine}
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine_t)
    else:
        allr = [mine_t]
    d4.free()
    o4.free()
    algo = n4 * L + 4 * n4
    r = {
        "workload": f"config4: {n4} fixed 4 KiB SSTable blocks per GPU ({n4 * L / GIB:.0f} GiB), rank r = blocks "
                    f"[r*{n4}, (r+1)*{n4}) of config 2's stream, device-resident",
        "value": round(world * n4 * L / GIB / (wall_max / a.steps), 2), "unit": "GiB/s",
        "ms_per_step": round(wall_max * 1e3 / a.steps, 4), "steps": a.steps, "records_per_gpu": n4,
        "kernel": "crc32_wring_kernel",
        "frac": round(algo / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "per_rank": allr,
    }
    g4 = golden_summaries().get("config4", {}).get("shard_summary_crc32", [])
    if n4 == (1 << 26) and world <= len(g4):
        r["summary_matches_oracle"] = [x["summary_crc32"] for x in allr] == g4[:world]
    return r


def main():
    a = parse()
    rc = relaunch(a)
    if rc is not None:
        sys.exit(rc)
    global torch, dist, _lib, Context, gen_zipf_lengths
    import torch  # first: liblsmck must bind to the HIP runtime torch loaded (lsm_storage_engine_amd/_lib.py)
    import torch.distributed as dist
    from lsm_storage_engine_amd import _lib
    from lsm_storage_engine_amd.device import Context, gen_zipf_lengths
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("LSMCK_BENCH_SHARE_GPU"):  # rehearsal of the N-rank path on a 1-GPU box
        local %= torch.cuda.device_count()
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(local)
    stream = torch.cuda.Stream(device=local)  # a real stream: the null stream's handle (0) means
    sptr = stream.cuda_stream                 # "the context's own stream" to liblsmck
    ctx = Context(local)
    if a.stream != 1:
        ctx.set_option("crc_stream", a.stream)

    cfg = resolve_config(a.config, world)
    seed = SEED[cfg]
    if cfg == 2:
        # N > 1: BASELINE config 4, 2^26 blocks per GPU (256 GiB; 2^26/N per rank
        # when the ranks share one GPU in a rehearsal, LSMCK_BENCH_SHARE_GPU)
        c4 = world > 1 or a.blocks_per_gpu == (1 << 26)
        share = os.environ.get("LSMCK_BENCH_SHARE_GPU") and world > 1
        nrec = a.blocks_per_gpu or (((1 << 26) // world if share else (1 << 26)) if world > 1 else (1 << 24))
        rec_len = 4096
        nbytes = nrec * rec_len
        byte_off = rank * nbytes  # this rank's shard of the global block stream
        if c4:
            cname = "config4" if nrec == (1 << 26) else f"config4 (reduced shard: {nrec} blocks per rank)"
            workload = (f"{cname}: {nrec} fixed 4 KiB SSTable blocks per GPU ({nbytes / GIB:.0f} GiB), "
                        f"rank r = blocks [r*{nrec}, (r+1)*{nrec}) of config 2's stream, device-resident")
        else:
            workload = f"config2: {nrec} fixed 4 KiB SSTable blocks per GPU ({nbytes / GIB:.0f} GiB), device-resident"
    elif cfg == 1:
        nrec = a.blocks_per_gpu or (1 << 20)
        rec_len = 256
        nbytes = nrec * rec_len
        byte_off = rank * nbytes
        workload = f"config1: {nrec} x 256 B WAL payloads per GPU, device-resident"
    else:
        nrec = a.blocks_per_gpu or (1 << 26)
        A = max(1, a.pack_align)
        gather = None
        if world > 1:
            def gather(x):
                xs = [None] * world
                dist.all_gather_object(xs, x)
                return xs
        offs, lens, nbytes, byte_off = config3_shard(gen_zipf_lengths, seed, nrec, rank, gather, a.wal_framed, A)
        shard = (f"; rank r = records [r*{nrec}, (r+1)*{nrec}) of one global stream, bytes at its global offset"
                 if world > 1 else "")
        if a.wal_framed:
            workload = (f"config3w: {nrec} mixed-length records per GPU (64 B-64 KiB, Zipf s=1.5) framed as wal.rs "
                        f"Insert records: a 13-byte header before every payload, unaligned ({nbytes / GIB:.1f} GiB "
                        f"image), device-resident{shard}")
        else:
            workload = (f"config3: {nrec} mixed-length records per GPU (64 B-64 KiB, Zipf s=1.5, packed, unaligned; "
                        f"{nbytes / GIB:.1f} GiB), device-resident{shard}")
        if A > 1:
            workload += f" [diagnostic: offsets aligned to {A} B]"
        if a.sorted:
            workload += " [LSMCK_SORTED: caller-asserted order, no device-side descriptor check]"

    sha = a.digest == "sha256"
    data = ctx.alloc(nbytes + 64)
    ctx.gen_stream(data.ptr, seed, byte_off, nbytes, sptr)
    out = ctx.alloc((32 if sha else 4) * nrec)
    if cfg != 3 and a.desc:  # diagnostic: the same fixed blocks as descriptors
        offs = np.arange(nrec, dtype=np.uint64) * np.uint64(rec_len)
        lens = np.full(nrec, rec_len, dtype=np.uint32)
        workload += " [diagnostic: descriptor entry point]"
    if cfg == 3 or a.desc:
        d_off, d_len = ctx.alloc(8 * nrec), ctx.alloc(4 * nrec)
        d_off.upload(offs)
        d_len.upload(lens)
        payload = int(lens.astype(np.uint64).sum())

        if sha:
            def step():
                ctx.sha256_device(data.ptr, d_off.ptr, d_len.ptr, nrec, out.ptr, sptr)
            sha_blocks = int(((lens.astype(np.uint64) + 9 + 63) // 64).sum())
        else:
            def step():
                ctx.crc32_device(data.ptr, d_off.ptr, d_len.ptr, nrec, out.ptr, sptr, sorted_span=a.sorted)
        algo_bytes = payload + 12 * nrec + (32 if sha else 4) * nrec
    else:
        payload = nbytes
        if sha:
            def step():
                ctx.sha256_fixed_device(data.ptr, rec_len, rec_len, nrec, out.ptr, sptr)
            sha_blocks = nrec * ((rec_len + 9 + 63) // 64)
        else:
            def step():
                ctx.crc32_fixed_device(data.ptr, rec_len, rec_len, nrec, out.ptr, sptr)
        algo_bytes = payload + (32 if sha else 4) * nrec
    torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    ctx.sync(sptr)
    torch.cuda.synchronize()

    ab = None
    if a.variants:
        # interleaved A/B rounds in ONE process (cdna_hip_programming.md 5.4 rule 24)
        vs = a.variants.split(",")
        ab = {v: [] for v in vs}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        defaults = {"crc_stream": 1, "crc_ablate": 0, "sha_pair": 1, "sha_bucket_shift": 2, "sha_bucket_from": 128,
                    "sha_short_blocks": 12}
        keys = {"s": "crc_stream", "a": "crc_ablate", "p": "sha_pair", "b": "sha_bucket_shift", "f": "sha_bucket_from",
                "t": "sha_short_blocks"}
        for _ in range(a.rounds):
            for v in vs:
                opts = dict(defaults)
                for part in ([] if v == "-" else v.split("+")):
                    m = re.fullmatch(r"([sapbft])(\d+)", part)
                    if not m:
                        raise SystemExit(f"bad variant {v!r}")
                    opts[keys[m.group(1)]] = int(m.group(2))
                for k, val in opts.items():
                    ctx.set_option(k, val)
                step()
                e0.record(stream)
                for _ in range(a.steps):
                    step()
                e1.record(stream)
                ctx.sync(sptr)
                ab[v].append(e0.elapsed_time(e1) / a.steps)
        for k, val in defaults.items():
            ctx.set_option(k, val)
        ab = {str(v): {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                       "GiBps_median": payload / GIB / (float(np.median(t)) * 1e-3)} for v, t in ab.items()}

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    ctx.sync(sptr)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    wall = t1 - t0
    ev_ms = ev0.elapsed_time(ev1) / a.steps
    t = torch.tensor([wall], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t[0])

    ms_per_step = wall_max * 1000.0 / a.steps
    total_payload = payload * world
    value = total_payload / GIB / (wall_max / a.steps)
    achieved_gbs = algo_bytes / (ev_ms * 1e-3) / 1e9
    # PMC traffic per launch from the committed profiles.  Config 4 (a shard of
    # fixed 4 KiB blocks per rank): measured on the 2^26-block shard; a reduced
    # shard (the shared-GPU rehearsal) scales it by its block count, since the
    # kernel's bytes are per block.  Other diagnostics have no committed traffic.
    c4 = cfg == 2 and not sha and not a.desc and (world > 1 or nrec == (1 << 26))
    if c4:
        t4 = traffic_from_profiles("config4")
        traffic = None if t4 is None else round(t4 * nrec / float(1 << 26), 1)
    else:
        cname = f"config{cfg}" + ("w" if a.wal_framed else "")
        wkey = None if (a.desc or a.pack_align > 1 or a.blocks_per_gpu) else f"{'sha256_' if sha else ''}{cname}"
        traffic = traffic_from_profiles(wkey)
    # every rank's own launch time (HIP events on its stream) and wall time
    mine_t = {"rank": rank, "launch_ms_hip_events": round(ev_ms, 4), "wall_ms_per_step": round(wall * 1e3 / a.steps, 4),
              "frac": round(algo_bytes / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine_t)
    else:
        per_rank = [mine_t]

    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64 counter stream generated in HBM (same bytes as oracle_gen_stream)",
        "config": {
            "workload": workload,
            "records_per_gpu": nrec,
            "payload_bytes_per_gpu": payload,
            "parallelism": f"record-sharded x{world}, no data-path collective",
            "checksum": "CRC-32/ISO-HDLC (crc::crc32::checksum_ieee)",
        },
        "hbm_frac_of_peak": round(value * GIB / 1e9 / world / HBM_PEAK_GBS, 4),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            # fixed records whose segment count divides 64 (configs 1, 2) run the
            # whole-tile ring kernel by default (lsmck_crc32.hip, LSMCK_DEFAULT_RING)
            # config 3 is packed with records >= 64 B: the stream kernel takes it
            "kernel": (("crc32_stream_kernel" if a.stream else "crc32_walk_kernel") if (cfg == 3 or a.desc)
                       else "crc32_wring_kernel"),
            "algorithmic_bytes_per_launch": algo_bytes,
            "launch_ms_hip_events": round(ev_ms, 4),
            # achieved and launch_ms are rank 0's; every rank's are under per_rank
            "launch_ms_min_max_over_ranks": [min(r["launch_ms_hip_events"] for r in per_rank),
                                             max(r["launch_ms_hip_events"] for r in per_rank)],
            "frac_min_over_ranks": min(r["frac"] for r in per_rank),
        },
        "per_rank": per_rank,
        "cpu_baseline": None,
        "hip_runtime": _lib._foreign_hip_runtime_loaded(),
    }
    if ab is not None:
        res["variants_ab"] = ab
    if sha:
        # SHA-256 is bound by int32 VALU issue, not HBM: one
        # compression = SHA_OPS_PER_BLOCK VALU lane-ops (count of the compression
        # loop's VALU instructions in the kernel ISA), chip peak 256 CU x 128
        # lane-ops/clk x 2.4 GHz = 78.6 T lane-ops/s (MI355X_MICROARCH.md:
        # 157.3 TFLOPS FP32 vector = 128 FMA lanes/clk/CU).
        ops = sha_blocks * SHA_OPS_PER_BLOCK
        res["config"]["checksum"] = "SHA-256 per record (sha2::Sha256, checksums.rs:20-38 applied per record)"
        res["roofline"] = {
            "bound": "valu",
            "achieved": round(ops / (ev_ms * 1e-3) / 1e12, 2),
            "peak": VALU_PEAK_TOPS,
            "unit": "T VALU issue slots/s (half-rate ops count 2)",
            "frac": round(ops / (ev_ms * 1e-3) / 1e12 / VALU_PEAK_TOPS, 4),
            "traffic": traffic,
            "kernel": "sha256_kernel",
            "compression_blocks_per_launch": sha_blocks,
            "slots_per_block": SHA_OPS_PER_BLOCK,
            "hbm_GBps": round(algo_bytes / (ev_ms * 1e-3) / 1e9, 1),
            "launch_ms_hip_events": round(ev_ms, 4),
        }
        res["hbm_frac_of_peak"] = round(algo_bytes / (ev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    # Host round trip (north_star: the path starts and ends in host memory):
    # a sample of the same records in pinned host memory, one synchronous
    # lsmck_crc32_batch* per step = H2D DMA + kernel + D2H, chunked and
    # double-buffered inside liblsmck.  Reported beside `value`, never as it.
    if rank == 0 and world == 1 and not a.no_host_roundtrip and not sha:
        if cfg == 3 or a.desc:
            hn = min(nrec, 1 << 21)
            hbytes = int(offs[hn - 1]) + int(lens[hn - 1])
        else:
            hn = min(nrec, (4 << 30) // rec_len)
            hbytes = hn * rec_len
        pb = ctx.alloc_pinned(hbytes)
        ctx.memcpy_d2h(pb.ptr, data.ptr, hbytes)
        if cfg == 3 or a.desc:
            hoff, hlen = offs[:hn].copy(), lens[:hn].copy()

            def hstep():
                return ctx.crc32(pb.array, hoff, hlen, pinned=True)
            hpay = int(hlen.astype(np.uint64).sum())
        else:
            def hstep():
                return ctx.crc32_fixed(pb.array, rec_len, rec_len, hn, pinned=True)
            hpay = hbytes
        hres = hstep()
        hsteps = 3
        th0 = time.perf_counter()
        for _ in range(hsteps):
            hres = hstep()
        th = (time.perf_counter() - th0) / hsteps
        res["host_roundtrip"] = {
            "value": round(hpay / GIB / th, 2), "unit": "GiB/s", "ms_per_step": round(th * 1e3, 2),
            "sample": f"first {hn} records ({hpay / GIB:.2f} GiB) in pinned host memory; "
                      "synchronous lsmck_crc32_batch* with LSMCK_HOST_PINNED (H2D DMA + kernel + D2H)",
            "matches_device_result": bool(np.array_equal(hres, out.download(np.uint32, count=hn))),
        }
        pb.free()

    # summary digest: CRC-32 of the little-endian output array
    # (CRCs, or the 32-B digests), for cross-run comparison; every rank's, for N > 1
    import zlib
    mine = "%08x" % zlib.crc32(out.download(np.uint8, count=(32 if sha else 4) * nrec).tobytes())
    if world > 1:
        allsum = [None] * world
        dist.all_gather_object(allsum, mine)
    else:
        allsum = [mine]
    if rank == 0:
        res["summary_crc32"] = allsum[0]
        for pr, sm in zip(res["per_rank"], allsum):
            pr["summary_crc32"] = sm
        gold = golden_summaries()
        if world > 1 or (cfg == 2 and nrec == (1 << 26)):
            res["rank_summaries_crc32"] = allsum
            # config 4 shards against the oracle's (tests/golden/make_summaries.py config4)
            g4 = gold.get("config4", {}).get("shard_summary_crc32", [])
            if cfg == 2 and not sha and nrec == (1 << 26) and world <= len(g4):
                res["summary_matches_oracle"] = allsum == g4[:world]
            # config 3's global-stream shards (make_summaries.py config3_shards; a
            # reduced shard of 2^20 records per rank: config3_shards_small)
            g3 = gold.get(CONFIG3_SHARDS.get(nrec, ""), {}).get("shard_summary_crc32", [])
            if cfg == 3 and not sha and not a.wal_framed and a.pack_align <= 1 and world <= len(g3):
                res["summary_matches_oracle"] = allsum == g3[:world]
        elif not a.blocks_per_gpu and a.pack_align <= 1:
            # against the oracle's full-size value (default layouts only)
            g = gold.get(f"config{cfg}" + ("w" if a.wal_framed and cfg == 3 else ""), {}).get(
                "summary_sha256" if sha else "summary_crc32")
            if g:
                res["summary_matches_oracle"] = res["summary_crc32"] == g

    # CPU baseline + parity of the same sample (rank 0, N = 1 only)
    if rank == 0 and world == 1 and not a.no_cpu_baseline and sha:
        from oracle import oracle as O  # the checker / baseline, never the measured path
        ns = min(nrec, a.cpu_sample_records or (1 << 16))
        if cfg == 3:
            send = int(offs[ns - 1]) + int(lens[ns - 1])
            host = O.gen_stream(seed, 0, send)
            so, sl = offs[:ns], lens[:ns]
        else:
            host = O.gen_stream(seed, byte_off, ns * rec_len)
            so = np.arange(ns, dtype=np.uint64) * np.uint64(rec_len)
            sl = np.full(ns, rec_len, dtype=np.uint32)
        tc0 = time.perf_counter()
        want = O.sha256_batch(host, so, sl, threads=1)
        tc = time.perf_counter() - tc0
        sbytes = int(sl.astype(np.uint64).sum())
        got = out.download(np.uint8, count=32 * ns).reshape(ns, 32)
        res["cpu_baseline"] = {
            "value": round(sbytes / GIB / tc, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {ns} records ({sbytes / GIB:.2f} GiB); oracle FIPS 180-4 SHA-256 (= sha2 0.10 "
                      "Sha256, scalar, no SHA-NI), 1 thread",
            "seconds": round(tc, 2),
            "gpu_matches_on_sample": bool(np.array_equal(got, np.asarray(want).reshape(ns, 32))),
        }
        # SURVEY 8d CPU rows (2) and (4): all host cores, and OpenSSL (hashlib; SHA-NI where the CPU has it)
        tc0 = time.perf_counter()
        O.sha256_batch(host, so, sl, threads=CPU_ALL_CORES)
        tall = time.perf_counter() - tc0
        import hashlib
        mv = memoryview(host)
        tc0 = time.perf_counter()
        for o, l in zip(so.tolist(), sl.tolist()):
            hashlib.sha256(mv[o:o + l]).digest()
        tossl = time.perf_counter() - tc0
        res["cpu_extra"] = {
            "oracle_all_cores": {"value": round(sbytes / GIB / tall, 3), "unit": "GiB/s", "cores": CPU_ALL_CORES},
            "openssl_hashlib_1_thread": {"value": round(sbytes / GIB / tossl, 3), "unit": "GiB/s", "cores": 1},
            "sample": "the cpu_baseline sample",
        }
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not sha:
        from oracle import oracle as O  # the checker / baseline, never the measured path
        if cfg == 3:
            ns = a.cpu_sample_records or (1 << 21)
            ns = min(ns, nrec)
            send = int(offs[ns - 1]) + int(lens[ns - 1])
            host = O.gen_stream(seed, 0, send)
            tc0 = time.perf_counter()
            want = O.crc32_batch(host, offs[:ns], lens[:ns], threads=1)
            tc = time.perf_counter() - tc0
            sbytes = int(lens[:ns].astype(np.uint64).sum())
            sample = f"first {ns} records of the same Zipf stream ({sbytes / GIB:.2f} GiB)"
        else:
            ns = a.cpu_sample_records or ((1 << 20) if cfg == 2 else (1 << 22))
            ns = min(ns, nrec)
            host = O.gen_stream(seed, byte_off, ns * rec_len)
            tc0 = time.perf_counter()
            want = O.crc32_fixed(host, rec_len, rec_len, ns, threads=1)
            tc = time.perf_counter() - tc0
            sbytes = ns * rec_len
            sample = f"first {ns} records of the same stream ({sbytes / GIB:.2f} GiB)"
        got = out.download(np.uint32, count=ns)
        res["cpu_baseline"] = {
            "value": round(sbytes / GIB / tc, 3),
            "unit": "GiB/s",
            "cores": 1,
            "kind": "port",
            "sample": sample + "; oracle Sarwate byte-at-a-time CRC-32 (= crc 1.x checksum_ieee), 1 thread",
            "seconds": round(tc, 2),
            "gpu_matches_on_sample": bool(np.array_equal(got, want)),
        }
        # SURVEY 8d CPU rows (2) and (3): all host cores (oracle), and zlib's crc32 (slicing / PCLMUL;
        # faster than, and not, the reference's algorithm; informational)
        so = offs[:ns] if cfg == 3 else np.arange(ns, dtype=np.uint64) * np.uint64(rec_len)
        sl = lens[:ns] if cfg == 3 else np.full(ns, rec_len, dtype=np.uint32)
        tc0 = time.perf_counter()
        if cfg == 3:
            O.crc32_batch(host, so, sl, threads=CPU_ALL_CORES)
        else:
            O.crc32_fixed(host, rec_len, rec_len, ns, threads=CPU_ALL_CORES)
        tall = time.perf_counter() - tc0
        import zlib
        mv = memoryview(host)
        tc0 = time.perf_counter()
        zl = [zlib.crc32(mv[o:o + l]) for o, l in zip(so.tolist(), sl.tolist())]
        tz = time.perf_counter() - tc0
        res["cpu_extra"] = {
            "oracle_all_cores": {"value": round(sbytes / GIB / tall, 3), "unit": "GiB/s", "cores": CPU_ALL_CORES},
            "zlib_1_thread": {"value": round(sbytes / GIB / tz, 3), "unit": "GiB/s", "cores": 1,
                              "matches": bool(np.array_equal(np.asarray(zl, dtype=np.uint32), want))},
            "sample": "the cpu_baseline sample",
        }
    # The kernel's own memory ceiling ("report against a measured
    # streaming-read peak from the build's own read-only kernel"): the same
    # kernel and launch with crc_ablate 3 -- payload loads only, no checksum,
    # no store -- on the same buffer, timed like the bench line.  Last: it
    # leaves `out` invalid, so every check of `out` above runs first.
    if rank == 0 and world == 1 and not sha and not a.no_stream_ceiling and ab is None:
        ctx.set_option("crc_ablate", 3)
        try:
            step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(5):
                step()
            e1.record(stream)
            ctx.sync(sptr)
            lms = e0.elapsed_time(e1) / 5
        finally:
            ctx.set_option("crc_ablate", 0)
        ceil_gbs = algo_bytes / (lms * 1e-3) / 1e9
        res["roofline"]["loads_only_ceiling"] = {
            "GBps": round(ceil_gbs, 1), "launch_ms": round(lms, 4),
            "frac_of_ceiling": round(achieved_gbs / ceil_gbs, 4),
            "how": "same kernel with crc_ablate 3: payload loads only (no checksum, no store), same buffer",
        }

    # BASELINE config 4 beside the config-3 line: the per-GPU fixed-block shard
    # (its own 1 -> N curve from the same runs), after config 3's buffers go
    if cfg == 3 and not sha and not a.no_config4:
        data.free()
        out.free()
        for b in (d_off, d_len):
            b.free()
        res["config4"] = config4_sub(a, ctx, stream, sptr, world, rank)

    if rank == 0:
        print(json.dumps(res), flush=True)
    ctx.sync(sptr)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
