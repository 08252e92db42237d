#!/bin/bash
# round 5: config 5 through the server (100 GiB), then Db::load restarts with 8 / 4 / 2 index-loading threads
set -o pipefail
O=gpurun_out/r05srv2; mkdir -p $O
timeout -k 10 1100 python3 -u tools/e2e_server.py --gib 100 --dir /dev/shm/lsm_e2e_server_r05 --load-ab 8,4,2 > $O/server.log 2>&1 || { echo "server failed"; tail -8 $O/server.log; exit 1; }
grep "^first start\|^restart\|^load index" $O/server.log | cut -c1-400
