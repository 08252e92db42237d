#!/bin/bash
# walking-kernel check: smoke, CRC/WAL/async GPU tests, config-3 bench walk vs tile map
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$R.log 2>&1; step smoke $?
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_async.py tests/test_gpu_crc.py tests/test_gpu_wal.py ${PYTEST_EXTRA} > gpurun_out/pytest_$R.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_$R.log; step pytest $rc
timeout -k 10 300 python3 bench.py --config 3 --steps 10 --no-cpu-baseline --no-host-roundtrip > gpurun_out/bench_${R}_c3_walk.log 2>&1; step bench_walk $?
tail -1 gpurun_out/bench_${R}_c3_walk.log
timeout -k 10 300 python3 bench.py --config 3 --steps 10 --no-cpu-baseline --no-host-roundtrip --walk 0 > gpurun_out/bench_${R}_c3_tile.log 2>&1; step bench_tile $?
tail -1 gpurun_out/bench_${R}_c3_tile.log
