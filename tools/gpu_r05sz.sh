#!/bin/bash
# round 5, last tree: config 5 through the server at 100 GiB (Db::load first start and restarts, compaction ticks)
set -o pipefail
O=gpurun_out/r05sz; mkdir -p $O
timeout -k 10 1100 python3 -u tools/e2e_server.py --gib 100 --dir /dev/shm/lsm_e2e_server_r05z --load-ab 3 > $O/server.log 2>&1 || { echo "server failed"; tail -8 $O/server.log; exit 1; }
grep "^first start\|^restart\|^load index\|^ticks" $O/server.log | cut -c1-330
