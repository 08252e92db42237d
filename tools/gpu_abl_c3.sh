#!/bin/bash
# config-3 stream kernel ablations, interleaved in one process (median ms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-abl}
timeout -k 10 600 python3 bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --variants ${VARIANTS:-c0,a8,a5,a4,a6,a2,a3} --rounds ${ROUNDS:-3} > gpurun_out/$T.log 2>&1; rc=$?
tail -1 gpurun_out/$T.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:round(v['median_ms'],3) for k,v in d['variants_ab'].items()})"
exit $rc
