#!/bin/bash
# fixed ring kernel tile orders: parity, then interleaved A/B on config 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_async.py > gpurun_out/pytest_$R.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$R.log; step pytest $rc
timeout -k 10 300 python3 bench.py --config 2 --steps 10 --no-cpu-baseline --no-host-roundtrip --variants c2,c2o1,c2o2,a3,a3o1,a3o2 --rounds 6 > gpurun_out/ab_order_${R}.log 2>&1; step ab_order $?
python3 -c "import json;d=json.loads(open('gpurun_out/ab_order_$R.log').read().strip().splitlines()[-1]);print(json.dumps(d['variants_ab'],indent=0))"
