#!/bin/bash
# round 5: where the compaction tick's batch goes (LSMCK_TREE_TRACE's summary line per verify): levels 0..3 of a
# 100 GiB tree through lsmck_checksums_verify_many, three ticks, and the whole tree once
set -o pipefail
O=gpurun_out/r05ts; mkdir -p $O
LSMCK_TREE_TRACE=1 timeout -k 10 1000 python3 -u tools/e2e_tree.py --gib 100 --reps 1 --tick 4,4,4 --cpu-sample-gib 0.1 --dir /dev/shm/lsm_e2e_r05ts > $O/tree.log 2>&1 || { echo "tree failed"; tail -8 $O/tree.log; exit 1; }
grep "^tick\|^rep\|^tree verify:" $O/tree.log
