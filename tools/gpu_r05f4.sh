#!/bin/bash
# round 5: why the lane-dense finish (D3) loses -- SQ counters of P1 and D3, config 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05f4; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_wt.so
B="python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_COUNT"
for N in P1 D3; do
  cp $L/ab/$N.so $L/liblsmck.so
  n=0
  for P in "$P1" "$P2"; do
    n=$((n+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/${N}_p$n -o p -- $B > $O/${N}_p$n.log 2>&1 || { echo "$N pass $n failed"; tail -5 $O/${N}_p$n.log; cp /tmp/liblsmck_wt.so $L/liblsmck.so; exit 1; }
  done
  python3 tools/pmc_table.py $O/${N}_p1 $O/${N}_p2 > $O/sq_table_$N.txt 2>&1
  echo "== $N"; grep -A20 "stream_kernel<0>" $O/sq_table_$N.txt | grep -v "^\[" | head -40
done
cp /tmp/liblsmck_wt.so $L/liblsmck.so
