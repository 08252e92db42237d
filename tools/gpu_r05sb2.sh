#!/bin/bash
# round 5: scan width / lanes a guess, second pass: config 3w sweeps of B1G16 and B2G8 (two scan blocks, eight lanes),
# then the hard logs (~1 MiB values, log of logs) on H3 / B1G8 / B2G8 at the automatic segment size
set -o pipefail
O=gpurun_out/r05sb2; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
for N in B1G16 B2G8 B1G8 H3; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --seg-sweep 786432,1048576,1572864,2097152 > $O/sweep_$N.log 2>&1 || { echo "sweep $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/sweep_$N.log; exit 1; }
  echo "$N zipf: $(tail -n 1 $O/sweep_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["records_on_device"]; print("default", r["ms_median"], {k: (v["ms_median"], v["repairs"], v["path"]) for k, v in r["seg_sweep"].items()})')"
done
for shape in mib logs; do
  for N in H3 B1G8 B2G8; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape $shape > $O/${shape}_$N.log 2>&1 || { echo "$shape $N failed"; cp /tmp/liblsmck_keep.so $L/liblsmck.so; tail -5 $O/${shape}_$N.log; exit 1; }
    echo "$N $shape: $(tail -n 1 $O/${shape}_$N.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("hbm", d["records_on_device"]["ms_median"], "repairs", d["seg_repairs"], "prepairs", d["seg_prepairs"], d["walk_path"])')"
  done
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
