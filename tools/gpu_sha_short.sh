#!/bin/bash
# SHA-256: the lean kernel for an ordered batch's short tail -- tests, then
# config 3 A/B over the block threshold (sha_short_blocks; t0 = off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03t}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sha.py -m gpu -q -rf -x --timeout 200 --timeout-method thread > gpurun_out/pytest_sha_$R.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_sha_$R.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u bench.py --digest sha256 --config 3 --steps 3 --warmup 1 --variants=${VARIANTS:--,t1,t2,t3,t4,t6} --rounds 3 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/ab_sha_short_$R.log 2>&1; rc=$?
tail -1 gpurun_out/ab_sha_short_$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get("variants_ab"), indent=0))'
exit $rc
