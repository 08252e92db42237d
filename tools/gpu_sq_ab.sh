#!/bin/bash
# SQ / GRBM counters of the stream kernel for each A/B library build
# (tools/build_ab.sh): one rocprofv3 --pmc pass per build over the config-3
# bench (3 steps), then tools/sq_summary.py per build.
#   LIBS="perm bop" ROUND=r06r [PMC="..."] bash tools/gpu_sq_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${ROUND:-r06}
mkdir -p $O
L=lsm_storage_engine_amd
PMC=${PMC:-"GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"}
cp $L/liblsmck.so /tmp/liblsmck_wt.so
for N in $LIBS; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -s KILL 240 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $O/sq_$N -o sq -- python3 bench.py --config ${CFG:-3} --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4 ${BENCH_EXTRA} > $O/sq_$N.log 2>&1 || { echo "pmc $N failed"; cp /tmp/liblsmck_wt.so $L/liblsmck.so; exit 1; }
  python3 tools/sq_summary.py $O/sq_$N crc32_stream_kernel > $O/sq_$N.txt 2>&1
  echo "== $N"; cat $O/sq_$N.txt
done
cp /tmp/liblsmck_wt.so $L/liblsmck.so
