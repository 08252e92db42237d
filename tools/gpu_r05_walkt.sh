#!/bin/bash
# round 5: kernel trace of the 97.8 GiB replay with compact records (SDMA read-back to a pinned array, then in HBM)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05kt; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/kt -o kt -- python3 tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 > $O/walbig_kt.log 2>&1 || { echo "traced replay failed"; tail -20 $O/walbig_kt.log; exit 1; }
python3 tools/kt_stats.py $O/kt > $O/kt_stats.txt
grep -E "replay" $O/walbig_kt.log | head -10
head -24 $O/kt_stats.txt
