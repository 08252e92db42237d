#!/bin/bash
# round 5: the last window's CRCs pushed at once (N0), and with the payload loads in chain order (N1):
# stream + CRC tests on both, then same-box A/B against H0 (configs 3 and 3w)
set -o pipefail
O=gpurun_out/r05f9; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
for N in N0 N1; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_crc.py -k "not multicontext" > $O/pytest_$N.log 2>&1 || { echo "pytest $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_$N.log; exit 1; }
  echo "$N: $(tail -n 1 $O/pytest_$N.log)"
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
LIBS="H0 N0 N1" ROUNDS=6 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
LIBS="H0 N0 N1" ROUNDS=3 CFG=3 BENCH_EXTRA=--wal-framed bash tools/gpu_ab_libs.sh > $O/ab_c3w.log 2>&1 || { cat $O/ab_c3w.log; exit 1; }
cat $O/ab_c3w.log
