#!/bin/bash
# The round's evidence in one GPU call: smoke, GPU parity, the default bench
# line (config 2) and config 3, the SHA-256 lines, rocprofv3 kernel-trace stats
# of each, and the PMC traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs).
# Every GPU step has its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1; step smoke $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_$R.log; step pytest $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${R}_c2.log 2>&1; step bench_c2 $?
tail -1 gpurun_out/bench_${R}_c2.log
timeout -k 10 400 python3 bench.py --config 3 --steps 10 > gpurun_out/bench_${R}_c3.log 2>&1; step bench_c3 $?
tail -1 gpurun_out/bench_${R}_c3.log
timeout -k 10 400 python3 bench.py --digest sha256 --steps 5 --warmup 1 > gpurun_out/bench_${R}_sha_c2.log 2>&1; step bench_sha_c2 $?
timeout -k 10 400 python3 bench.py --digest sha256 --config 3 --steps 5 --warmup 1 > gpurun_out/bench_${R}_sha_c3.log 2>&1; step bench_sha_c3 $?
for W in "2" "3" "2 --digest sha256"; do
  set -- $W; CFG=$1; shift; TAG=c$CFG${1:+_sha}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_$TAG -o kt -- python3 bench.py --config $CFG "$@" --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip > gpurun_out/kt_${R}_$TAG.log 2>&1; step kt_$TAG $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_${TAG}_$C -o pmc -- python3 bench.py --config $CFG "$@" --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip > gpurun_out/pmc_${R}_${TAG}_$C.log 2>&1; step pmc_${TAG}_$C $?
  done
  KEY=config$CFG; [ -n "$1" ] && KEY=sha256_config$CFG
  python3 tools/pmc_summary.py gpurun_out/pmc_${R}_${TAG}_FETCH_SIZE gpurun_out/pmc_${R}_${TAG}_WRITE_SIZE $KEY > gpurun_out/pmc_summary_${R}_$TAG.json
done
python3 tools/kt_stats.py gpurun_out/kt_${R}_c2 gpurun_out/kt_${R}_c3 gpurun_out/kt_${R}_c2_sha > gpurun_out/kt_stats_$R.txt
cat gpurun_out/kt_stats_$R.txt
