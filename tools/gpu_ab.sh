#!/bin/bash
# Parity for every variant, then interleaved A/B of kernel variants in one
# process per workload, then PMC counter passes on the default variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf --timeout 600 > gpurun_out/pytest_gpu_$R.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu_$R.log
[ $rc -le 1 ] || exit $rc
for CFG in ${AB_CONFIGS:-2 3}; do
  timeout -k 10 400 python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --variants ${VARIANTS:-c1,c2,c4} --rounds 3 > gpurun_out/ab_${R}_c$CFG.log 2>&1
  rc=$?; echo "ab config$CFG rc=$rc"; tail -1 gpurun_out/ab_${R}_c$CFG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('variants_ab'))"
  [ $rc -eq 0 ] || exit $rc
done
[ -n "$SKIP_PMC" ] && exit 0
P1="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VMEM_RD,SQ_INST_LEVEL_VMEM,SQ_LDS_DATA_FIFO_FULL,SQ_LDS_CMD_FIFO_FULL,GRBM_COUNT"
i=0
for P in $P1 $P2; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/sq_${R}_p$i -o sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sq_${R}_p$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
