#!/bin/bash
# round 5: HBM bytes of the dependent header loads -- FETCH_SIZE of the chase microbenchmark (known load counts) to
# calibrate the 16-byte random-load case, then FETCH_SIZE / WRITE_SIZE per dispatch of the WAL replay's kernels
set -o pipefail
O=gpurun_out/r05pw; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/chase_f -o pmc -- ./tools/microbench_chase 1600 1300 > $O/chase_f.log 2>&1 || { echo "chase pmc failed"; tail -5 $O/chase_f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/wal_f -o pmc -- python3 tools/wal_replay_big.py --steps 1 --compact 1 --device-recs 1 > $O/wal_f.log 2>&1 || { echo "wal fetch pmc failed"; tail -5 $O/wal_f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/wal_w -o pmc -- python3 tools/wal_replay_big.py --steps 1 --compact 1 --device-recs 1 > $O/wal_w.log 2>&1 || { echo "wal write pmc failed"; tail -5 $O/wal_w.log; exit 1; }
ls -R $O | head -30
