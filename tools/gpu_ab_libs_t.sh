#!/bin/bash
# Same-box A/B of library builds (tools/build_ab.sh) with each build's stream
# kernel tests first (tests/test_gpu_stream.py, plus TESTS if set); then
# ROUNDS interleaved bench rounds on config $CFG.  LIBS="A B ..." required.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_wt.so
restore() { cp /tmp/liblsmck_wt.so $L/liblsmck.so; }
for N in $LIBS; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py ${TESTS} -m gpu -q -rf -x --timeout 200 --timeout-method thread > gpurun_out/abt_${N}.log 2>&1; rc=$?
  echo "$N tests: $(tail -1 gpurun_out/abt_${N}.log)"
  [ $rc -eq 0 ] || { restore; exit $rc; }
done
for r in $(seq 1 ${ROUNDS:-3}); do
  for N in $LIBS; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 200 python3 -u bench.py --config ${CFG:-3} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling ${BENCH_EXTRA} > gpurun_out/abl_${N}_$r.log 2>&1 || { echo "bench $N failed"; restore; exit 1; }
    echo "$N round $r: $(tail -1 gpurun_out/abl_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["launch_ms_hip_events"], d.get("summary_matches_oracle"))')"
  done
done
restore
