#!/bin/bash
# round 5: lane-dense finish (D1, -DLSMCK_STREAM_DEFER=1) -- stream tests on D1, then same-box A/B against H0
set -o pipefail
O=gpurun_out/r05f; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
cp $L/ab/D1.so $L/liblsmck.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_crc.py -k "not multicontext" > $O/pytest_stream_D1.log 2>&1 || { echo "pytest failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_stream_D1.log; exit 1; }
cp /tmp/liblsmck_keep.so $L/liblsmck.so
tail -n 2 $O/pytest_stream_D1.log
LIBS="H0 D1" ROUNDS=5 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
LIBS="H0 D1" ROUNDS=3 CFG=3 BENCH_EXTRA=--wal-framed bash tools/gpu_ab_libs.sh > $O/ab_c3w.log 2>&1 || { cat $O/ab_c3w.log; exit 1; }
cat $O/ab_c3w.log
