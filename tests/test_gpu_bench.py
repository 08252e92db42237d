"""bench.py's N-rank path and BASELINE config 4 on the GPU.

* `python bench.py --gpus 2` (no launcher) must start two ranks itself
  (torch.distributed.run as a child process), report n_gpus 2 and the config-3
  workload -- rank r = records [r*n, (r+1)*n) of one global stream -- and
  every rank's shard must match the oracle's digest (committed:
  tests/golden/summaries.json config3_shards_small); its config-4 sub-line
  likewise (digests computed here).  The two ranks share the box's one GPU
  (LSMCK_BENCH_SHARE_GPU=1) on reduced shards.  --config 2 keeps the
  config-4 shard as the main line.
* Config 4's per-GPU shard at full size (2^26 x 4 KiB = 256 GiB, rank 0's
  blocks [0, 2^26) of config 2's stream) through the C ABI, against the
  oracle's summary digest (tests/golden/make_summaries.py config4).
"""
import json
import os
import subprocess
import sys
import zlib

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED2 = 0x5EED0002


def _oracle_shard_summary(rank, nrec, threads=16):
    data = O.gen_stream(SEED2, rank * nrec * 4096, nrec * 4096)
    crc = O.crc32_fixed(data, 4096, 4096, nrec, threads=threads)
    return "%08x" % zlib.crc32(crc.astype("<u4").tobytes())


def _bench2(*args, gpus=2, timeout=300):
    env = dict(os.environ, LSMCK_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "3",
                        "--warmup", "1", *args], cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])


@pytest.mark.gpu
def test_bench_gpus2_config3_global_stream():
    """The default N-rank line: config 3 on both ranks, each its own segment of
    one global stream (2^20 records per rank here), digests equal to the
    oracle's; the config-4 sub-line's shards too."""
    nrec, n4 = 1 << 20, 1 << 18
    r = _bench2("--blocks-per-gpu", str(nrec), "--c4-blocks", str(n4))
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    assert r["config"]["workload"].startswith("config3")
    assert r["config"]["records_per_gpu"] == nrec
    with open(os.path.join(ROOT, "tests", "golden", "summaries.json")) as f:
        g = json.load(f)["config3_shards_small"]
    assert r["rank_summaries_crc32"] == g["shard_summary_crc32"][:2]
    assert r["summary_matches_oracle"] is True
    # value = both ranks' payload over the slowest rank's time
    pay = sum(g["shard_bytes"][:2])
    assert abs(r["value"] - pay / 2**30 / (r["ms_per_step"] * 1e-3)) / r["value"] < 0.01
    c4 = r["config4"]
    assert c4["records_per_gpu"] == n4
    assert [p["summary_crc32"] for p in c4["per_rank"]] == [_oracle_shard_summary(k, n4) for k in range(2)]
    assert abs(c4["value"] - 2 * n4 * 4096 / 2**30 / (c4["ms_per_step"] * 1e-3)) / c4["value"] < 0.01


@pytest.mark.gpu
def test_bench_gpus8_rehearsal():
    """The 8-rank line before the driver's 8-GPU node runs it: eight ranks on
    the box's one GPU (LSMCK_BENCH_SHARE_GPU=1), reduced shards.  Every
    rank's config-3 shard -- records [r*2^20, (r+1)*2^20) of one global
    stream -- equals the committed oracle digest, every rank's config-4 shard
    the oracle's (computed here), and value is all ranks' payload over the
    slowest rank's time."""
    nrec, n4 = 1 << 20, 1 << 18
    r = _bench2("--blocks-per-gpu", str(nrec), "--c4-blocks", str(n4), gpus=8, timeout=600)
    assert r["n_gpus"] == 8 and r["scaling"] == "weak"
    assert r["config"]["workload"].startswith("config3")
    with open(os.path.join(ROOT, "tests", "golden", "summaries.json")) as f:
        g = json.load(f)["config3_shards_small"]
    assert len(g["shard_summary_crc32"]) == 8
    assert r["rank_summaries_crc32"] == g["shard_summary_crc32"]
    assert r["summary_matches_oracle"] is True
    pay = sum(g["shard_bytes"][:8])
    assert abs(r["value"] - pay / 2**30 / (r["ms_per_step"] * 1e-3)) / r["value"] < 0.01
    c4 = r["config4"]
    assert [p["summary_crc32"] for p in c4["per_rank"]] == [_oracle_shard_summary(k, n4) for k in range(8)]
    assert abs(c4["value"] - 8 * n4 * 4096 / 2**30 / (c4["ms_per_step"] * 1e-3)) / c4["value"] < 0.01


@pytest.mark.gpu
def test_bench_gpus2_launches_two_ranks():
    nrec = 1 << 18  # 1 GiB per rank
    env = dict(os.environ, LSMCK_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "2",
                        "--blocks-per-gpu", str(nrec), "--steps", "3", "--warmup", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 2
    assert r["config"]["workload"].startswith("config4")
    assert r["config"]["records_per_gpu"] == nrec
    assert r["scaling"] == "weak"
    want = [_oracle_shard_summary(k, nrec) for k in range(2)]
    assert r["rank_summaries_crc32"] == want
    # the N > 1 line is evaluable: PMC traffic (config 4's, scaled to the
    # reduced shard) and every rank's own launch time
    assert r["roofline"]["traffic"] is not None and r["roofline"]["traffic"] > 0
    assert [p["rank"] for p in r["per_rank"]] == [0, 1]
    lo, hi = r["roofline"]["launch_ms_min_max_over_ranks"]
    assert 0 < lo <= hi
    assert all(0 < p["frac"] < 1 for p in r["per_rank"])
    assert [p["summary_crc32"] for p in r["per_rank"]] == want
    # value = both ranks' payload over the slowest rank's time
    assert abs(r["value"] - 2 * nrec * 4096 / 2**30 / (r["ms_per_step"] * 1e-3)) / r["value"] < 0.01


def test_bench_default_workload_is_config3():
    """Every N defaults to BASELINE config 3 (north_star's 64 B-64 KiB records
    at 1, 2, 4 and 8 GPUs): the 1 -> N curve is like for like."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.resolve_config(0, 1) == 3
    assert bench.resolve_config(0, 8) == 3
    assert bench.resolve_config(2, 8) == 2


def test_bench_world_size_mismatch_fails():
    """Under a launcher, WORLD_SIZE must equal --gpus (checked before any GPU call)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr


@pytest.mark.gpu
def test_config4_rank0_shard_full_size(ctx):
    """2^26 x 4 KiB = 256 GiB on one GPU, every CRC checked through the summary digest."""
    with open(os.path.join(ROOT, "tests", "golden", "summaries.json")) as f:
        want = json.load(f)["config4"]["shard_summary_crc32"][0]
    n = 1 << 26
    d = ctx.alloc(n * 4096)
    out = ctx.alloc(4 * n)
    try:
        ctx.gen_stream(d.ptr, SEED2, 0, n * 4096)
        ctx.crc32_fixed_device(d.ptr, 4096, 4096, n, out.ptr)
        ctx.sync()
        crc = out.download(np.uint32)
        assert "%08x" % zlib.crc32(crc.astype("<u4").tobytes()) == want
        # and a spread sample against the oracle record by record
        idx = np.linspace(0, n - 1, 512).astype(np.int64)
        for i in idx[::64]:
            blk = O.gen_stream(SEED2, int(i) * 4096, 4096)
            assert crc[i] == O.crc32(blk)
    finally:
        d.free()
        out.free()
