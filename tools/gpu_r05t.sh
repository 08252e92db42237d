#!/bin/bash
# round 5: the whole-tree verify cycling through three pinned slots instead of two (tree_stages A/B),
# tree tests first, then a 16 GiB tree (e2e_tree.py --stages 2,3, interleaved)
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree.py tests/test_server.py -m gpu > $O/pytest_tree.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_tree.log; exit 1; }
tail -n 1 $O/pytest_tree.log
timeout -k 10 900 python3 -u tools/e2e_tree.py --gib 16 --reps 2 --stages 2,3 --dir /dev/shm/lsm_e2e_r05t > $O/tree.log 2>&1 || { echo "tree failed"; tail -8 $O/tree.log; exit 1; }
grep "^stages\|^rep" $O/tree.log
