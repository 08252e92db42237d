#!/bin/bash
# round 5: compact WAL records + SDMA read-back -- GPU tests, then the 97.8 GiB replay A/B
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wal_compact.py tests/test_gpu_wal.py > $O/pytest_wal.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_wal.log; exit 1; }
tail -3 $O/pytest_wal.log
for args in "--compact 1" "--compact 0" "--compact 1 --dma-engines 0" "--compact 0 --dma-engines 0" "--compact 1 --device-recs 1 --steps 3"; do
  echo "== $args" >> $O/walbig.log
  timeout -k 10 240 python -u tools/wal_replay_big.py --steps 5 $args >> $O/walbig.log 2>&1 || { echo "walbig failed: $args"; tail -20 $O/walbig.log; exit 1; }
done
grep -E "^==|ms_median" $O/walbig.log | cut -c1-400
