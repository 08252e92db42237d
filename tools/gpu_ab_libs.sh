#!/bin/bash
# Same-box A/B of library builds (tools/build_ab.sh): for each round, each
# build in turn runs the bench on config $CFG (default 3); prints the ms per step.
#   LIBS="A B" ROUNDS=3 CFG=3 [BENCH_EXTRA=--wal-framed] bash tools/gpu_ab_libs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_wt.so
for r in $(seq 1 ${ROUNDS:-3}); do
  for N in $LIBS; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 200 python3 -u bench.py --config ${CFG:-3} --steps ${BENCH_STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling ${BENCH_EXTRA} > gpurun_out/abl_${N}_$r.log 2>&1 || { echo "bench $N failed"; cp /tmp/liblsmck_wt.so $L/liblsmck.so; exit 1; }
    echo "$N round $r: $(tail -1 gpurun_out/abl_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["launch_ms_hip_events"])')"
  done
done
cp /tmp/liblsmck_wt.so $L/liblsmck.so
