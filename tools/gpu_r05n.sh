#!/bin/bash
# round 5: segments sized to the walk kernel's residency (N2) against powers of two (H2):
# WAL GPU tests on N2, then the 97.8 GiB logs (config 3w, ~1 MiB values, log of logs), records in HBM and to the host
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
cp $L/ab/N2.so $L/liblsmck.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest_wal_N2.log 2>&1 || { echo "pytest N2 failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_wal_N2.log; exit 1; }
tail -n 1 $O/pytest_wal_N2.log
for shape in zipf mib logs; do
  for r in 1 2; do
    for N in H2 N2; do
      cp $L/ab/$N.so $L/liblsmck.so
      timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape $shape > $O/walbig_${shape}_${N}_$r.log 2>&1 || { echo "walbig $shape $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/walbig_${shape}_${N}_$r.log; exit 1; }
      echo "$shape $N round $r: $(tail -n 1 $O/walbig_${shape}_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("host", d["ms_median"], "hbm", d["records_on_device"]["ms_median"], "segments", d["segments"], "repairs", d["seg_repairs"], "prepairs", d["seg_prepairs"], d["walk_path"])')"
    done
  done
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
