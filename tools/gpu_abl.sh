#!/bin/bash
# Interleaved stream-kernel ablations on config 3 (bench --variants), after the
# stream kernel's own GPU tests.  VARIANTS / ROUNDS / TAG / BENCH_EXTRA from the env.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-abl}
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_stream.py -m gpu -q -rf -x --timeout 200 --timeout-method thread > gpurun_out/pytest_stream_$T.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_stream_$T.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python3 -u bench.py --config 3 --steps ${STEPS:-5} --warmup 2 --variants=${VARIANTS:--,a3,a5,a9,a10,a4} --rounds ${ROUNDS:-3} --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling ${BENCH_EXTRA} > gpurun_out/ab_$T.log 2>&1; rc=$?
tail -1 gpurun_out/ab_$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get("variants_ab"), indent=0))'
exit $rc
