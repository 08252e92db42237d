#!/bin/bash
# The round's evidence in one GPU call: smoke, GPU parity, the default bench
# line (config 2) and config 3, rocprofv3 kernel-trace stats of both, and the
# PMC traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs) of both.
# Every GPU step has its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1; step smoke $?
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf --timeout 600 > gpurun_out/pytest_gpu_$R.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_$R.log; step pytest $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${R}_c2.log 2>&1; step bench_c2 $?
tail -1 gpurun_out/bench_${R}_c2.log
timeout -k 10 400 python3 bench.py --config 3 --steps 10 > gpurun_out/bench_${R}_c3.log 2>&1; step bench_c3 $?
tail -1 gpurun_out/bench_${R}_c3.log
for CFG in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_c$CFG -o kt -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-host-roundtrip > gpurun_out/kt_${R}_c$CFG.log 2>&1; step kt_c$CFG $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_c${CFG}_$C -o pmc -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip > gpurun_out/pmc_${R}_c${CFG}_$C.log 2>&1; step pmc_c${CFG}_$C $?
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${R}_c${CFG}_FETCH_SIZE gpurun_out/pmc_${R}_c${CFG}_WRITE_SIZE config$CFG > gpurun_out/pmc_summary_${R}_c$CFG.json
done
python3 tools/kt_stats.py gpurun_out/kt_${R}_c2 gpurun_out/kt_${R}_c3 > gpurun_out/kt_stats_$R.txt
cat gpurun_out/kt_stats_$R.txt
