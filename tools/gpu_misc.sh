#!/bin/bash
# Stream-kernel deferred-push A/B (config 3), then rocprofv3 kernel stats of
# the default bench command itself (same steps as the bench line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02m}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_$R.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_$R.log; step pytest $rc
timeout -k 10 400 python3 bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip --variants ${VARIANTS:-c0,c0t2} --rounds 4 > gpurun_out/ab_$R.log 2>&1; step ab $?
tail -1 gpurun_out/ab_$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d.get('variants_ab'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${R}_default -o kt -- python3 bench.py > gpurun_out/kt_${R}_default.log 2>&1; step kt_default $?
tail -1 gpurun_out/kt_${R}_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_ms_hip_events'])"
python3 tools/kt_stats.py gpurun_out/kt_${R}_default | head -6
