#!/bin/bash
# round 5: stream-kernel event words re-coded once per tile -- stream tests, then same-box A/B
set -o pipefail
O=gpurun_out/r05b2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_crc.py -k "not multicontext" > $O/pytest_stream.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_stream.log; exit 1; }
tail -n 2 $O/pytest_stream.log
LIBS="H0 E1" ROUNDS=4 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
LIBS="H0 E1" ROUNDS=3 CFG=3 BENCH_EXTRA=--wal-framed bash tools/gpu_ab_libs.sh > $O/ab_c3w.log 2>&1 || { cat $O/ab_c3w.log; exit 1; }
cat $O/ab_c3w.log
