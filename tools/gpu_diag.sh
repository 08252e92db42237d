#!/bin/bash
# Memory-path diagnosis of the CRC kernels: per-kernel time split (kernel
# trace) and TA/TCP/UTCL1/TCC counters for the fixed (config 2) and the
# descriptor (config 3) kernels, one small counter group per rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
if [ -z "$SKIP_MB" ] && [ -x tools/microbench_loads ]; then
  timeout -k 10 120 ./tools/microbench_loads ${MB_GB:-64} > gpurun_out/mbl_$R.log 2>&1 || exit $?
  cat gpurun_out/mbl_$R.log
fi
[ -z "$SKIP_KT" ] && for CFG in ${DIAG_CONFIGS:-3 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${R}_c$CFG -o kt -- python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_${R}_c$CFG.log 2>&1
  rc=$?; echo "kt config$CFG rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
PMCG=${PMC_GROUPS:-"TCP_UTCL1_TRANSLATION_MISS,TCP_UTCL1_REQUEST,TCP_TOTAL_CACHE_ACCESSES,TCP_TCC_READ_REQ TA_TA_BUSY,TA_ADDR_STALLED_BY_TC_CYCLES,TA_DATA_STALLED_BY_TC_CYCLES,TD_TC_STALL TCP_PENDING_STALL_CYCLES,TCP_READ_TAGCONFLICT_STALL_CYCLES,TCP_TCR_TCP_STALL_CYCLES,TCP_TCP_TA_DATA_STALL_CYCLES TCC_HIT,TCC_MISS,TCC_EA0_RDREQ,TCC_TAG_STALL"}
for CFG in ${DIAG_CONFIGS:-3 2}; do
  i=0
  for G in $PMCG; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $G --kernel-trace --output-format csv -d gpurun_out/diag_${R}_c${CFG}_g$i -o d -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/diag_${R}_c${CFG}_g$i.log 2>&1
    rc=$?; echo "pmc config$CFG group$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/pmc_table.py gpurun_out/diag_${R}_c* > gpurun_out/diag_$R.txt
cat gpurun_out/diag_$R.txt
