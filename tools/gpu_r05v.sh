#!/bin/bash
# round 5: the product tree after one-block scan steps and eight guess lanes -- WAL GPU tests, then the 97.8 GiB logs
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wal.py tests/test_gpu_wal_compact.py tests/test_gpu_crc.py -k "wal or config3w" > $O/pytest_wal.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_wal.log; exit 1; }
tail -n 1 $O/pytest_wal.log
for shape in zipf mib logs; do
  timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 5 --compact 1 --device-recs 1 --shape $shape > $O/walbig_$shape.log 2>&1 || { echo "walbig $shape failed"; tail -5 $O/walbig_$shape.log; exit 1; }
  echo "$shape: $(tail -n 1 $O/walbig_$shape.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("host", d["ms_median"], "hbm", d["records_on_device"]["ms_median"], "repairs", d["seg_repairs"], "prepairs", d["seg_prepairs"], d["walk_path"])')"
done
