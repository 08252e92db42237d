#!/usr/bin/env python3
"""Summary digests of the BASELINE configs at full size ("Summary
digest = CRC-32 of the output array, for cross-run comparison").

For each config every record's digest is computed on the CPU by the oracle
(oracle/: Sarwate CRC-32, FIPS 180-4 SHA-256; pinned against zlib and hashlib
by tests/test_oracle.py) over the same splitmix64 byte stream the GPU generates
(oracle_gen_stream == gen_stream_kernel), in 1 GiB chunks on a thread pool so
host memory stays small.  The summary is zlib.crc32 of the output array: the
little-endian u32 CRCs, or the 32-byte SHA-256 digests in record order.
tests/test_gpu_crc.py / test_gpu_sha.py compare the GPU's full-size outputs
with these values; bench.py prints the GPU's as "summary_crc32".

  config 1: 2^20 x 256 B, seed 0x5EED0001
  config 2: 2^24 x 4096 B, seed 0x5EED0002
  config 3: 2^26 Zipf(1.5) records of 64 B - 64 KiB packed back to back,
            lengths from the seed, bytes from the same seed
  config 3w: config 3's records framed as wal.rs Insert records: record i's
            payload starts 13 bytes (its header) after record i-1 ends
            (off_i = 13 (i+1) + sum of the earlier lengths); bytes from the
            same seed over the whole image, CRC-32 only (bench.py --wal-framed)
  config 4: 8 per-GPU shards of 2^26 x 4096 B (256 GiB each) of config 2's
            block stream (seed 0x5EED0002): shard r = blocks [r*2^26, (r+1)*2^26),
            CRC-32 only (bench.py's config4 sub-measurement: rank r checksums shard r)
  config3_shards: 8 per-GPU shards of ONE global config-3 stream: shard r =
            records [r*2^26, (r+1)*2^26) (lengths from the counter-based
            generator at record r*2^26), packed, its bytes at the global
            offset where shard r-1 ends (bench.py --gpus N: rank r); shard 0
            is config 3 itself.  config3_shards_small: the same with 2^20
            records per shard (the shared-GPU rehearsal in test_gpu_bench.py)

Run:  python3 tests/golden/make_summaries.py [crc|sha|all|config4|config3w|config3_shards|config3_shards_small]
      (updates summaries.json here)
"""
import concurrent.futures as cf
import json
import os
import sys
import time
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

CHUNK = 1 << 30
THREADS = int(os.environ.get("THREADS", "8"))
OUT = os.path.join(HERE, "summaries.json")


def _digest(data, off, ln, sha):
    if sha:
        return np.asarray(O.sha256_batch(data, off, ln, threads=1), dtype=np.uint8).tobytes()
    return O.crc32_batch(data, off, ln, threads=1).astype("<u4").tobytes()


def _chunks(offs, lens):
    """record ranges [r0, r1) of about CHUNK payload bytes"""
    ends = offs + lens.astype(np.uint64)
    r0, n = 0, len(offs)
    while r0 < n:
        r1 = max(int(np.searchsorted(ends, offs[r0] + np.uint64(CHUNK), side="right")), r0 + 1)
        yield r0, r1
        r0 = r1


def summary(seed, offs, lens, sha, byte_off=0):
    def job(rng):
        r0, r1 = rng
        base = int(offs[r0])
        data = O.gen_stream(seed, byte_off + base, int(offs[r1 - 1]) + int(lens[r1 - 1]) - base)
        return _digest(data, offs[r0:r1] - np.uint64(base), lens[r0:r1], sha)
    crc = 0
    with cf.ThreadPoolExecutor(THREADS) as ex:  # ctypes calls release the GIL
        for part in ex.map(job, list(_chunks(offs, lens))):
            crc = zlib.crc32(part, crc)
    return "%08x" % crc


def layout_wal(lens, header=13):
    """payload descriptors of records framed with a `header`-byte header each"""
    offs = np.full(len(lens), header, dtype=np.uint64)  # payload i+1 starts len[i] + header after payload i
    offs[1:] += lens[:-1].astype(np.uint64)
    return np.cumsum(offs, dtype=np.uint64), lens


def layout(cfg):
    if cfg == 1:
        n, L = 1 << 20, 256
    elif cfg == 2:
        n, L = 1 << 24, 4096
    else:
        lens = O.gen_zipf_lengths(0x5EED0003, 1 << 26)
        offs = np.zeros(len(lens), dtype=np.uint64)
        np.cumsum(lens[:-1].astype(np.uint64), out=offs[1:])
        return offs, lens
    return np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, dtype=np.uint32)


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    res["method"] = ("oracle digest per record (1 GiB chunks), zlib.crc32 of the output array "
                     "(LE u32 CRCs / 32-B SHA-256 digests)")
    t0 = time.time()
    if what == "config3w":
        offs, lens = layout_wal(O.gen_zipf_lengths(0x5EED0003, 1 << 26))
        e = res.setdefault("config3w", {})
        e.update({"records": len(offs), "payload_bytes": int(lens.astype(np.uint64).sum()),
                  "image_bytes": int(offs[-1]) + int(lens[-1]), "seed": hex(0x5EED0003), "header_bytes": 13,
                  "summary_crc32": summary(0x5EED0003, offs, lens, False)})
        print("config3w", e, round(time.time() - t0, 1), flush=True)
        with open(OUT, "w") as f:
            json.dump(res, f, indent=1)
            f.write("\n")
        return
    if what in ("config3_shards", "config3_shards_small"):
        n = 1 << (26 if what == "config3_shards" else 20)
        e = res.setdefault(what, {})
        e.update({"records_per_shard": n, "seed": hex(0x5EED0003),
                  "layout": "shard r = records [r*n, (r+1)*n) of one global packed config-3 stream, "
                            "bytes at the stream offset where shard r-1 ends"})
        shards = e.setdefault("shard_summary_crc32", [])
        e.setdefault("shard_bytes", [])
        byte_off = sum(e["shard_bytes"])
        for r in range(len(shards), 8):
            lens = O.gen_zipf_lengths(0x5EED0003, n, first=r * n)
            offs = np.zeros(n, dtype=np.uint64)
            np.cumsum(lens[:-1].astype(np.uint64), out=offs[1:])
            nbytes = int(offs[-1]) + int(lens[-1])
            if r == 0 and n == (1 << 26) and res.get("config3", {}).get("summary_crc32"):
                shards.append(res["config3"]["summary_crc32"])  # shard 0 is config 3 itself
            else:
                shards.append(summary(0x5EED0003, offs, lens, False, byte_off=byte_off))
            e["shard_bytes"].append(nbytes)
            byte_off += nbytes
            print(what, r, shards[-1], nbytes, round(time.time() - t0, 1), flush=True)
            with open(OUT, "w") as f:
                json.dump(res, f, indent=1)
                f.write("\n")
        return
    if what == "config4":
        n, L = 1 << 26, 4096
        offs, lens = np.arange(n, dtype=np.uint64) * np.uint64(L), np.full(n, L, dtype=np.uint32)
        e = res.setdefault("config4", {})
        e.update({"records_per_shard": n, "record_bytes": L, "seed": hex(0x5EED0002),
                  "shard_byte_offset": "rank * 2^38 (shard r = blocks [r*2^26, (r+1)*2^26) of config 2's stream)"})
        shards = e.setdefault("shard_summary_crc32", [])
        for r in range(len(shards), 8):
            shards.append(summary(0x5EED0002, offs, lens, False, byte_off=r * n * L))
            print("config4 shard", r, shards[-1], round(time.time() - t0, 1), flush=True)
            with open(OUT, "w") as f:
                json.dump(res, f, indent=1)
                f.write("\n")
        return
    for cfg in (1, 2, 3):
        seed = 0x5EED0000 + cfg
        offs, lens = layout(cfg)
        e = res.setdefault(f"config{cfg}", {})
        e.update({"records": len(offs), "payload_bytes": int(offs[-1]) + int(lens[-1]), "seed": hex(seed)})
        if what in ("crc", "all"):
            e["summary_crc32"] = summary(seed, offs, lens, False)
        if what in ("sha", "all") and cfg != 1:
            e["summary_sha256"] = summary(seed, offs, lens, True)
        print(f"config{cfg}", e, round(time.time() - t0, 1), flush=True)
        with open(OUT, "w") as f:
            json.dump(res, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
