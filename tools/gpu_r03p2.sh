#!/bin/bash
# Round-3 later evidence: the stream kernel's tests (incl. the check's
# alignment/position cases), the official bench lines, traces and PMC, then
# the B/C library A/B (pre-decoded event words) on configs 3 and 3w.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py -m gpu -q -rf -x --timeout 200 --timeout-method thread > gpurun_out/pytest_stream_r03p.log 2>&1 || { tail -20 gpurun_out/pytest_stream_r03p.log; exit 1; }
tail -1 gpurun_out/pytest_stream_r03p.log
ROUND=r03p STEPS="bench c3w c2 kt kt3w c3pmc c3wpmc" bash tools/gpu_r03.sh || exit 1
[ -n "$LIBS" ] || exit 0
bash tools/gpu_ab_libs_t.sh || exit 1
NOTEST=1 BENCH_EXTRA=--wal-framed bash tools/gpu_ab_libs_t.sh
