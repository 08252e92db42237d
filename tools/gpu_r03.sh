#!/bin/bash
# Round-3 evidence in one GPU call.  Steps are picked by STEPS (space list):
#   c4pmc smoke quick pytest bench c3w c2 kt kt3w c3wpmc c3pmc sha shaab shakt shapmc wal (run in this order)
# Every GPU step has its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03}
STEPS=${STEPS:-"smoke pytest bench kt"}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has c4pmc; then  # config 4's 2^26-block shard (the N > 1 line's traffic)
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_c4_$C -o pmc -- python3 bench.py --config 2 --blocks-per-gpu 67108864 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/pmc_${R}_c4_$C.log 2>&1; step pmc_c4_$C $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${R}_c4_FETCH_SIZE gpurun_out/pmc_${R}_c4_WRITE_SIZE config4 > gpurun_out/pmc_summary_${R}_c4.json
  python3 tools/pmc_merge.py "$R (gpurun_out/pmc_${R}_c4_*)" gpurun_out/pmc_summary_${R}_c4.json
  cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_${R}.json
fi
if has smoke; then
  timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1; step smoke $?
fi
if has quick; then  # the stream kernel's own tests first (a fast signal)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stream.py tests/test_gpu_wal.py -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pytest_quick_$R.log 2>&1; rc=$?
  tail -15 gpurun_out/pytest_quick_$R.log; step quick $rc
fi
if has pytest; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_$R.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu_$R.log; step pytest $rc
fi
if has bench; then  # the driver's default line: config 3
  timeout -k 10 400 python3 bench.py > gpurun_out/bench_${R}_c3.log 2>&1; step bench_c3 $?
  tail -1 gpurun_out/bench_${R}_c3.log
fi
if has c3w; then  # config 3 framed as a WAL image (13-byte headers between the payloads)
  timeout -k 10 400 python3 bench.py --wal-framed > gpurun_out/bench_${R}_c3w.log 2>&1; step bench_c3w $?
  tail -1 gpurun_out/bench_${R}_c3w.log
fi
if has c2; then
  timeout -k 10 400 python3 bench.py --config 2 > gpurun_out/bench_${R}_c2.log 2>&1; step bench_c2 $?
  tail -1 gpurun_out/bench_${R}_c2.log
fi
if has kt; then  # kernel-trace stats of the default bench command
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_c3 -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-roundtrip > gpurun_out/kt_${R}_c3.log 2>&1; step kt_c3 $?
  python3 tools/kt_stats.py gpurun_out/kt_${R}_c3 > gpurun_out/kt_stats_${R}_c3.txt
  cat gpurun_out/kt_stats_${R}_c3.txt
fi
if has kt3w; then  # kernel-trace stats of config 3 framed as a WAL image
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_c3w -o kt -- python3 bench.py --wal-framed --steps 10 --warmup 2 --no-cpu-baseline --no-host-roundtrip > gpurun_out/kt_${R}_c3w.log 2>&1; step kt_c3w $?
  python3 tools/kt_stats.py gpurun_out/kt_${R}_c3w > gpurun_out/kt_stats_${R}_c3w.txt
  cat gpurun_out/kt_stats_${R}_c3w.txt
fi
if has c3wpmc; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_c3w_$C -o pmc -- python3 bench.py --wal-framed --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/pmc_${R}_c3w_$C.log 2>&1; step pmc_c3w_$C $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${R}_c3w_FETCH_SIZE gpurun_out/pmc_${R}_c3w_WRITE_SIZE config3w > gpurun_out/pmc_summary_${R}_c3w.json
fi
if has c3pmc; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_c3_$C -o pmc -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/pmc_${R}_c3_$C.log 2>&1; step pmc_c3_$C $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${R}_c3_FETCH_SIZE gpurun_out/pmc_${R}_c3_WRITE_SIZE config3 > gpurun_out/pmc_summary_${R}_c3.json
fi
if has sha; then
  timeout -k 10 400 python3 bench.py --digest sha256 --config 3 --steps 5 --warmup 1 > gpurun_out/bench_${R}_sha_c3.log 2>&1; step bench_sha_c3 $?
  tail -1 gpurun_out/bench_${R}_sha_c3.log
fi
if has shaab; then  # SHA-256 config 3: the pair kernel against its compute-only ablation (sha_pair 2) and single blocks
  timeout -k 10 600 python3 bench.py --digest sha256 --config 3 --steps 3 --warmup 1 --variants=-,p2,p3,p0 --rounds 3 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/ab_${R}_sha_c3.log 2>&1; step ab_sha_c3 $?
  tail -1 gpurun_out/ab_${R}_sha_c3.log
fi
if has shakt; then  # kernel-trace stats of SHA-256 config 3 (the order sort and the hash kernel)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_sha_c3 -o kt -- python3 bench.py --digest sha256 --config 3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/kt_${R}_sha_c3.log 2>&1; step kt_sha_c3 $?
  python3 tools/kt_stats.py gpurun_out/kt_${R}_sha_c3 > gpurun_out/kt_stats_${R}_sha_c3.txt
  cat gpurun_out/kt_stats_${R}_sha_c3.txt
fi
if has shapmc; then  # SHA-256 config 3 HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_sha_c3_$C -o pmc -- python3 bench.py --digest sha256 --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/pmc_${R}_sha_c3_$C.log 2>&1; step pmc_sha_c3_$C $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${R}_sha_c3_FETCH_SIZE gpurun_out/pmc_${R}_sha_c3_WRITE_SIZE sha256_config3 > gpurun_out/pmc_summary_${R}_sha_c3.json
fi
if has wal; then  # host WAL replay phases (LSMCK_WAL_TRACE) and the registered-upload A/B
  LSMCK_WAL_TRACE=1 timeout -k 10 300 python3 tools/wal_diag.py > gpurun_out/wal_diag_${R}.log 2>&1; step wal_diag $?
  tail -30 gpurun_out/wal_diag_${R}.log
fi
if has walkt; then  # kernel trace of the WAL replay (host image and device image)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_wal -o kt -- python3 tools/wal_kt.py > gpurun_out/kt_${R}_wal.log 2>&1; step kt_wal $?
  tail -1 gpurun_out/kt_${R}_wal.log
  python3 tools/kt_stats.py gpurun_out/kt_${R}_wal > gpurun_out/kt_stats_${R}_wal.txt
  cat gpurun_out/kt_stats_${R}_wal.txt
fi
echo "== done"
