#!/bin/bash
# stream kernel parity (small cases + config-3 full-size summary), then the
# config-3 ablation A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-sc}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_stream.py tests/test_gpu_crc.py -m gpu -x -q -k "${KSEL:-stream or packed or boundary or config3 or allocation or ineligible or host_batches or variants}" --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$T.log; [ $rc -eq 0 ] || exit $rc
TAG=abl_$T bash tools/gpu_abl_c3.sh
