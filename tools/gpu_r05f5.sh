#!/bin/bash
# round 5: lane-dense finish, third try: O3 (D3 + payload loads in chain order: the chain start's
# wait no longer covers the window reload) -- stream tests on O3, then A/B H0 / P1 / OP (P1 + order) / O3
set -o pipefail
O=gpurun_out/r05f5; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
for N in O3; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py > $O/pytest_stream_$N.log 2>&1 || { echo "pytest $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_stream_$N.log; exit 1; }
  echo "$N: $(tail -n 1 $O/pytest_stream_$N.log)"
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
LIBS="H0 P1 OP O3" ROUNDS=4 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
