#!/bin/bash
# PMC passes for the roofline "traffic" field: FETCH_SIZE and WRITE_SIZE in
# SEPARATE passes (their TCC slots do not fit one pass on gfx950), kernel-trace
# only alongside them, never sys/runtime trace.  Then summarise per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_counters_$R.txt 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_$C -o pmc -- python3 bench.py $ARGS > gpurun_out/pmc_${R}_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc_${R}_FETCH_SIZE gpurun_out/pmc_${R}_WRITE_SIZE "${WORKLOAD:-config2}" > gpurun_out/pmc_summary_$R.json
cat gpurun_out/pmc_summary_$R.json
