#!/bin/bash
# Instruction-fetch counters (one group per rocprofv3 run) of the config-3
# stream kernel and the config-2 ring kernel: I-cache requests / hits / misses
# and the instruction-fetch latency (SQ_IFETCH_LEVEL / SQ_IFETCH).
#   ROUND=r03d bash tools/gpu_icache.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03}
G1="SQC_ICACHE_REQ,SQC_ICACHE_HITS,SQC_ICACHE_MISSES,SQC_ICACHE_MISSES_DUPLICATE"
G2="SQ_IFETCH,SQ_IFETCH_LEVEL,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_BUSY_CYCLES"
for RUN in "c3:--config 3" "c2:--config 2"; do
  NAME=${RUN%%:*}; ARGS=${RUN#*:}
  i=0
  for G in $G1 $G2; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d gpurun_out/ic_${R}_${NAME}_g$i -o s -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/ic_${R}_${NAME}_g$i.log 2>&1
    rc=$?; echo "icache $NAME group$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/pmc_table.py gpurun_out/ic_${R}_* > gpurun_out/ic_$R.txt
cat gpurun_out/ic_$R.txt
