#!/bin/bash
# round 5, last tree: the server's index load with the sorted-insert hint -- tree + server GPU tests, then config 5
# through the server at 100 GiB (Db::load first start and restarts, compaction ticks)
set -o pipefail
O=gpurun_out/r05sx; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree.py tests/test_server.py -m gpu > $O/pytest_tree.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_tree.log; exit 1; }
tail -n 1 $O/pytest_tree.log
timeout -k 10 1100 python3 -u tools/e2e_server.py --gib 100 --dir /dev/shm/lsm_e2e_server_r05x --load-ab 2 > $O/server.log 2>&1 || { echo "server failed"; tail -8 $O/server.log; exit 1; }
grep "^first start\|^restart\|^load index\|^ticks" $O/server.log | cut -c1-330
