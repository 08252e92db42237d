#!/bin/bash
# round 5: large pinned buffers as registered huge pages -- the GPU suite, then config 5 through the server
set -o pipefail
O=gpurun_out/r05hp; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "suite failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 1100 python3 -u tools/e2e_server.py --gib 100 --dir /dev/shm/lsm_e2e_server_r05 --load-ab 2 > $O/server.log 2>&1 || { echo "server failed"; tail -8 $O/server.log; exit 1; }
grep "^first start\|^restart\|^load index\|^ticks" $O/server.log | cut -c1-330
