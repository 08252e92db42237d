#!/bin/bash
# round 5: parallel repair rounds of the segment walk; the hard logs at 1 GiB (tests) and 97.8 GiB; 8-rank rehearsal
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest_wal.log 2>&1 || { echo "pytest wal failed"; grep -E "FAIL|Error|assert" $O/pytest_wal.log | head -20; tail -5 $O/pytest_wal.log; exit 1; }
tail -n 2 $O/pytest_wal.log
timeout -k 10 700 python -u -m pytest -x -v --timeout 650 --timeout-method thread tests/test_gpu_bench.py -k gpus8 > $O/pytest_gpus8.log 2>&1 || { echo "pytest gpus8 failed"; tail -30 $O/pytest_gpus8.log; exit 1; }
tail -n 2 $O/pytest_gpus8.log
for sh in mib logs; do
  timeout -k 10 400 python -u tools/wal_replay_big.py --shape $sh --steps 2 --compact 1 --device-recs 1 > $O/walbig_$sh.log 2>&1 || { echo "walbig $sh failed"; tail -20 $O/walbig_$sh.log; exit 1; }
  grep -E "replay|log of logs" $O/walbig_$sh.log | head -12
  tail -n 1 $O/walbig_$sh.log | cut -c1-700
done
