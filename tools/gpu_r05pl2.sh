#!/bin/bash
# round 5: the placement kernel with three window buffers (no copy of a window in flight), unconditional slot loads, the record index base read once (PL0 before, PL1 after)
set -o pipefail
O=gpurun_out/r05pl2; mkdir -p $O
L=lsm_storage_engine_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest_wal.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_wal.log; exit 1; }
tail -n 1 $O/pytest_wal.log
cp $L/liblsmck.so /tmp/liblsmck_keep.so
for shape in zipf mib logs; do
  for r in 1 2; do
    for N in PL0 PL1; do
      cp $L/ab/$N.so $L/liblsmck.so
      timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape $shape > $O/${shape}_${N}_$r.log 2>&1 || { echo "walbig $shape $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/${shape}_${N}_$r.log; exit 1; }
      echo "$shape $N round $r: $(tail -n 1 $O/${shape}_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("host", d["ms_median"], "hbm", d["records_on_device"]["ms_median"], "repairs", d["seg_repairs"], d["walk_path"], d["summary_matches_oracle"], d["records_on_device"]["summary_matches_oracle"])')"
    done
  done
done
for N in PL0 PL1; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$N -o kt -- python3 tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 > $O/kt_$N.log 2>&1 || { echo "trace $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/kt_$N.log; exit 1; }
  grep -h "wal_seg_place\|wal_seg_walk_group\|crc32_stream_kernel" $O/kt_$N/kt_kernel_stats.csv | cut -c1-160
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
