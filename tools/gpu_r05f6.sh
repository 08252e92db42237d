#!/bin/bash
# round 5: lane-dense finish, where O3 loses: Q4 (no block multiply), Q5 (no shift-byte writes); both invalid
set -o pipefail
O=gpurun_out/r05f6; mkdir -p $O
LIBS="OP O3 Q4 Q5" ROUNDS=2 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
