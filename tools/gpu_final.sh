#!/bin/bash
# Round-end evidence on the final tree: smoke, the whole GPU suite, the
# full-size device WAL replay rate, the default bench line and its kernel trace.
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
echo "== done"
