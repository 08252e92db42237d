#!/bin/bash
# round 5: the compaction tick's batch (levels 0..3 of a 100 GiB tree through lsmck_checksums_verify_many):
# threads reading the checksum files (tree_json_threads) and files in flight (tree_active_files), interleaved
set -o pipefail
O=gpurun_out/${OUT:-r05tk}; mkdir -p $O
timeout -k 10 1000 python3 -u tools/e2e_tree.py --gib 100 --reps 1 --tick 2,4,4:16384,4:32768 --cpu-sample-gib 0.1 --dir /dev/shm/lsm_e2e_r05tk > $O/tree.log 2>&1 || { echo "tree failed"; tail -8 $O/tree.log; exit 1; }
grep "^tick\|^rep" $O/tree.log
