#!/bin/bash
# round 5: the segment walk on the logs it was not tuned for (97.8 GiB): ~1 MiB values, a log of logs
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
for sh in mib logs; do
  timeout -k 10 400 python -u tools/wal_replay_big.py --shape $sh --steps 2 --compact 1 --device-recs 1 > $O/walbig_$sh.log 2>&1 || { echo "walbig $sh failed"; tail -20 $O/walbig_$sh.log; exit 1; }
  grep -E "replay|log of logs" $O/walbig_$sh.log | head -12
  tail -n 1 $O/walbig_$sh.log | cut -c1-600
done
