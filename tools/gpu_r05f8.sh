#!/bin/bash
# round 5: the lane-dense finish builds' loss -- instruction-fetch counters of OP, O3, Q4 (config 3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05f8; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_wt.so
G1="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
G2="SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for N in OP O3 Q4; do
  cp $L/ab/$N.so $L/liblsmck.so
  i=0
  for G in "$G1" "$G2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $O/${N}_g$i -o s -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4 > $O/${N}_g$i.log 2>&1 || { echo "$N g$i failed"; tail -5 $O/${N}_g$i.log; cp /tmp/liblsmck_wt.so $L/liblsmck.so; exit 1; }
  done
  python3 tools/pmc_table.py $O/${N}_g1 $O/${N}_g2 > $O/ic_$N.txt
done
cp /tmp/liblsmck_wt.so $L/liblsmck.so
for N in OP O3 Q4; do echo "== $N"; grep -A12 "stream_kernel<0>" $O/ic_$N.txt | grep -v "^\[" | grep -v "^--" ; done
