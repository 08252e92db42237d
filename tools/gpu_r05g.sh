#!/bin/bash
# round 5: the later-start rule's scan window (kLaterScan): config 3w traced, then the hard shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest.log 2>&1 || { echo pytest failed; tail -20 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 > $O/walbig_kt.log 2>&1 || { echo "traced replay failed"; tail -20 $O/walbig_kt.log; exit 1; }
python3 tools/kt_stats.py $O/kt > $O/kt_stats.txt
grep -E "^replay" $O/walbig_kt.log | head -10
head -12 $O/kt_stats.txt
for args in "--shape zipf" "--shape mib" "--shape logs"; do
  echo "== $args"
  timeout -k 10 400 python -u tools/wal_replay_big.py $args --steps 3 --compact 1 --device-recs 1 > $O/walbig.log 2>&1 || { echo "walbig $args failed"; tail -20 $O/walbig.log; exit 1; }
  cat $O/walbig.log >> $O/walbig_all.log
  grep -E "^replay" $O/walbig.log | tail -4
done
