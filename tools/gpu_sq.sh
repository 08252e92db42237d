#!/bin/bash
# SQ counter passes (one group per rocprofv3 run) for CRC kernel variants:
# where a kernel's wave time goes (VALU, LDS, VMEM waits, in-flight level).
# usage: ROUND=r01x SQ_RUNS="name:args;name:args" bash tools/gpu_sq.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
G1="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INST_LEVEL_VMEM,SQ_ACTIVE_INST_VMEM,SQ_INSTS_SMEM,GRBM_COUNT"
IFS=';' read -ra RUNS <<< "${SQ_RUNS:-c2fixed:--config 2 --variants a3,c2;c2desc:--config 2 --desc --variants a3,c2}"
for RUN in "${RUNS[@]}"; do
  NAME=${RUN%%:*}; ARGS=${RUN#*:}
  i=0
  for G in $G1 $G2; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d gpurun_out/sq_${R}_${NAME}_g$i -o s -- python3 bench.py $ARGS --rounds 1 --steps 2 --warmup 1 --no-cpu-baseline --no-host-roundtrip > gpurun_out/sq_${R}_${NAME}_g$i.log 2>&1
    rc=$?; echo "sq $NAME group$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/pmc_table.py gpurun_out/sq_${R}_* > gpurun_out/sq_$R.txt
cat gpurun_out/sq_$R.txt
