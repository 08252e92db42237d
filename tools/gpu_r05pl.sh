#!/bin/bash
# round 5: the placement kernel's slot loads two windows ahead (P1) against one window at a time (P0):
# WAL GPU tests on P1, then the 97.8 GiB config-3w replay alternating builds, and its kernel trace on P1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05pl; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
cp $L/ab/P1.so $L/liblsmck.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest_wal_P1.log 2>&1 || { echo "pytest P1 failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_wal_P1.log; exit 1; }
tail -n 1 $O/pytest_wal_P1.log
for r in 1 2; do
  for N in P0 P1; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 5 --compact 1 --device-recs 1 > $O/walbig_${N}_$r.log 2>&1 || { echo "walbig $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/walbig_${N}_$r.log; exit 1; }
    echo "$N round $r: $(tail -n 1 $O/walbig_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("host", d["ms_median"], "hbm", d["records_on_device"]["ms_median"])')"
  done
done
for N in P0 P1; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$N -o kt -- python3 tools/wal_replay_big.py --steps 2 --compact 1 --device-recs 1 > $O/kt_$N.log 2>&1 || { echo "kt $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; exit 1; }
  python3 tools/kt_stats.py $O/kt_$N > $O/kt_stats_$N.txt 2>&1
  grep "seg_place\|walk_group" $O/kt_stats_$N.txt
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
