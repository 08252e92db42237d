#!/bin/bash
# round 5: the walk by the group's lanes through a shared window (LSMCK_SEG_WALK_WINDOW: 16-byte pieces a lane loads;
# 0 = lane 0 walks alone): WAL GPU tests on WW2, then A/B over the 97.8 GiB logs, records in HBM
set -o pipefail
O=gpurun_out/r05ww; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
cp $L/ab/WW2.so $L/liblsmck.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest_wal_WW2.log 2>&1 || { echo "pytest WW2 failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_wal_WW2.log; exit 1; }
tail -n 1 $O/pytest_wal_WW2.log
for shape in zipf mib; do
  for r in 1 2; do
    for N in WW0 WW1 WW2 WW4; do
      cp $L/ab/$N.so $L/liblsmck.so
      timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape $shape > $O/${shape}_${N}_$r.log 2>&1 || { echo "walbig $shape $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/${shape}_${N}_$r.log; exit 1; }
      echo "$shape $N round $r: $(tail -n 1 $O/${shape}_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("host", d["ms_median"], "hbm", d["records_on_device"]["ms_median"], "repairs", d["seg_repairs"], d["walk_path"])')"
    done
  done
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
