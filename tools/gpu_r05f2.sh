#!/bin/bash
# round 5: lane-dense finish, isolating its loss: H0 base, P1 (base, last window pushed at once),
# D1 (lane-dense finish), D2 (D1 with every shift 0: no LDS bank conflicts; results invalid)
set -o pipefail
O=gpurun_out/r05f2; mkdir -p $O
LIBS="H0 P1 D1 D2" ROUNDS=3 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
