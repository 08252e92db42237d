#!/bin/bash
# round 5: 16-byte staged records (W1) against 32 (H1): WAL GPU tests on W1, then the 97.8 GiB
# config-3w replay (compact records, to a pinned host array and in HBM), alternating builds;
# then the segment-size sweep on W1 (config 3w and the ~1 MiB-values log, records in HBM)
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
cp $L/ab/W1.so $L/liblsmck.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py > $O/pytest_wal_W1.log 2>&1 || { echo "pytest W1 failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -30 $O/pytest_wal_W1.log; exit 1; }
tail -n 1 $O/pytest_wal_W1.log
for r in 1 2; do
  for N in H1 W1; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 5 --compact 1 --device-recs 1 > $O/walbig_${N}_$r.log 2>&1 || { echo "walbig $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/walbig_${N}_$r.log; exit 1; }
    echo "$N round $r: $(tail -n 1 $O/walbig_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("host", d["ms_median"], "hbm", d["records_on_device"]["ms_median"])')"
  done
done
cp $L/ab/W1.so $L/liblsmck.so
timeout -k 10 400 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --seg-sweep 524288,1048576,2097152,4194304 > $O/sweep_zipf.log 2>&1 || { echo "zipf sweep failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/sweep_zipf.log; exit 1; }
tail -n 1 $O/sweep_zipf.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("zipf", d["ms_median"], d["records_on_device"]["seg_sweep"])'
timeout -k 10 400 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape mib --seg-sweep 524288,1048576,2097152,4194304 > $O/sweep_mib.log 2>&1 || { echo "mib sweep failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/sweep_mib.log; exit 1; }
tail -n 1 $O/sweep_mib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mib", d["ms_median"], d["records_on_device"]["seg_sweep"])'
cp /tmp/liblsmck_keep.so $L/liblsmck.so
