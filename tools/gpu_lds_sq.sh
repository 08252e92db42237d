#!/bin/bash
# LDS lookup-rate microbench, then SQ counter passes of the config-3 stream
# kernel and the config-2 ring kernel (instructions per tile, issue stalls).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/microbench_lds > gpurun_out/mb_lds.log 2>&1; rc=$?; cat gpurun_out/mb_lds.log; [ $rc -eq 0 ] || exit $rc
ROUND=r02s SQ_RUNS="c3stream:--config 3;c2ring:--config 2" bash tools/gpu_sq.sh
