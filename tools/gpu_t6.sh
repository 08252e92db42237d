#!/bin/bash
# tree verify + server GPU tests, then config 5 end to end (tools/e2e_server.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_tree.py tests/test_server.py > gpurun_out/pytest_tree_server_$R.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_tree_server_$R.log; step pytest $rc
timeout -k 10 700 python3 tools/e2e_server.py --gib ${GIB:-2} --ops ${OPS:-50000} > gpurun_out/e2e_server_$R.json 2> gpurun_out/e2e_server_$R.log; rc=$?
tail -2 gpurun_out/e2e_server_$R.log; tail -1 gpurun_out/e2e_server_$R.json; step e2e $rc
