#!/bin/bash
# round 5: does the stream kernel's LDS allocation alone slow it? OP with 1 KiB (L1) / 2 KiB (L2) more LDS, unused
set -o pipefail
O=gpurun_out/r05f7; mkdir -p $O
LIBS="OP L1 L2" ROUNDS=2 CFG=3 bash tools/gpu_ab_libs.sh > $O/ab_c3.log 2>&1 || { cat $O/ab_c3.log; exit 1; }
cat $O/ab_c3.log
