#!/bin/bash
# loopback server: GPU tests, then a small end-to-end run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_server.py > gpurun_out/pytest_server_$R.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_server_$R.log; step pytest $rc
timeout -k 10 600 python3 tools/e2e_server.py --gib ${GIB:-2} --ops ${OPS:-50000} > gpurun_out/e2e_server_$R.json 2> gpurun_out/e2e_server_$R.log; rc=$?
tail -3 gpurun_out/e2e_server_$R.log; tail -1 gpurun_out/e2e_server_$R.json; step e2e $rc
