#!/bin/bash
# round 5: lane-dense finish, second try -- stream tests on D3 and P3, then same-box A/B:
# H0 base, P1 (last window pushed at once), P3 (P1 + short-record loads consumed in their path),
# C3 (base + consumed), D3 (lane-dense finish + consumed)
set -o pipefail
O=gpurun_out/r05f3; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
for N in D3 P3; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py > $O/pytest_stream_$N.log 2>&1 || { echo "pytest $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_stream_$N.log; exit 1; }
  echo "$N: $(tail -n 1 $O/pytest_stream_$N.log)"
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
LIBS="H0 P1 P3 C3 D3" ROUNDS=3 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
