#!/bin/bash
# Round-end evidence on the final tree: smoke, the whole GPU suite, the
# full-size device WAL replay rate, the default bench line, its kernel trace
# and the config-3 PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03z}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1; step smoke $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$R.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$R.log; step pytest $rc
LSMCK_WAL_TRACE=1 timeout -k 10 400 python3 tools/wal_replay_big.py --steps 3 > gpurun_out/wal_replay_big_$R.json 2> gpurun_out/wal_replay_big_$R.log; rc=$?
tail -6 gpurun_out/wal_replay_big_$R.log; cat gpurun_out/wal_replay_big_$R.json; step wal_big $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${R}_c3.log 2>&1; step bench_c3 $?
tail -1 gpurun_out/bench_${R}_c3.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_c3 -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-roundtrip > gpurun_out/kt_${R}_c3.log 2>&1; step kt_c3 $?
python3 tools/kt_stats.py gpurun_out/kt_${R}_c3 > gpurun_out/kt_stats_${R}_c3.txt; cat gpurun_out/kt_stats_${R}_c3.txt
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_c3_$C -o pmc -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/pmc_${R}_c3_$C.log 2>&1; step pmc_c3_$C $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_${R}_c3_FETCH_SIZE gpurun_out/pmc_${R}_c3_WRITE_SIZE config3 > gpurun_out/pmc_summary_${R}_c3.json; cat gpurun_out/pmc_summary_${R}_c3.json
echo "== done"
