#!/bin/bash
# round 5: the walk kernel's occupancy against its scan width: scan blocks per step 4 (H3, 123 VGPRs, 4 waves/SIMD),
# 2 (B2, 90 VGPRs, 5), 1 (B1, 63 VGPRs, 8; B1G8: eight lanes a guess); 97.8 GiB config-3w log, records in HBM,
# segments 512 KiB / 1 / 2 MiB
set -o pipefail
O=gpurun_out/r05sb; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
for N in H3 B1 B1G8 B2; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --seg-sweep 524288,1048576,2097152 > $O/sweep_$N.log 2>&1 || { echo "sweep $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/sweep_$N.log; exit 1; }
  echo "$N: $(tail -n 1 $O/sweep_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["records_on_device"]; print("default", r["ms_median"], {k: (v["ms_median"], v["repairs"], v["path"]) for k, v in r["seg_sweep"].items()})')"
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
