#!/bin/bash
# round 5: the top level verified beside the lower levels' listing (tree_overlap): tree + server tests,
# then a 16 GiB tree A/B (e2e_tree.py --overlap 0,2048, interleaved)
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree.py tests/test_server.py -m gpu > $O/pytest_tree.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_tree.log; exit 1; }
tail -n 1 $O/pytest_tree.log
timeout -k 10 900 python3 -u tools/e2e_tree.py --gib 16 --reps 2 --overlap 0,2048 --dir /dev/shm/lsm_e2e_r05o > $O/tree.log 2>&1 || { echo "tree failed"; tail -8 $O/tree.log; exit 1; }
grep "^overlap\|^rep" $O/tree.log
