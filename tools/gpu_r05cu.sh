#!/bin/bash
# round 5: the config-3 stream pass on fewer workgroups than CUs (LSMCK_CUS), the data for running the WAL walk
# beside it on CUs of its own
set -o pipefail
O=gpurun_out/r05cu; mkdir -p $O
for r in 1 2; do
  for C in 256 248 240 224; do
    LSMCK_CUS=$C timeout -k 10 200 python3 bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4 > $O/c3_${C}_$r.log 2>&1 || { echo "bench $C failed"; tail -5 $O/c3_${C}_$r.log; exit 1; }
    echo "CUs $C round $r: $(grep '^{' $O/c3_${C}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"], d["summary_matches_oracle"])')"
  done
done
