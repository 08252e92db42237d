#!/bin/bash
# SQ wave-time breakdown (one rocprofv3 --pmc pass of 8 SQ counters per workload):
# where the checksum kernels' wave cycles go (parked on waitcnt, issue-stalled, active).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
for W in "2" "3" "2 --digest sha256"; do
  set -- $W; CFG=$1; shift; TAG=c$CFG${1:+_sha}
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/sq_$TAG -o sq -- python3 bench.py --config $CFG "$@" --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip > gpurun_out/sq_$TAG.log 2>&1 || exit $?
  echo "== $TAG ok"
done
