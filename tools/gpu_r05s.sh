#!/bin/bash
# round 5: SHA-256's effective clock (GRBM_GUI_ACTIVE / 8 / kernel time) and VALU issue on
# configs 2 and 3, beside the CRC stream kernel's (MI355X_MICROARCH.md "DVFS give-back")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for C in 2 3; do
  B="python3 bench.py --config $C --digest sha256 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4"
  timeout -k 10 200 $B > $O/bench_c$C.log 2>&1 || { echo "bench c$C failed"; tail -5 $O/bench_c$C.log; exit 1; }
  tail -n 1 $O/bench_c$C.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("roofline"))'
  timeout -s KILL 150 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/c${C}_p1 -o p -- $B > $O/c${C}_p1.log 2>&1 || { echo "pmc c$C failed"; tail -5 $O/c${C}_p1.log; exit 1; }
  python3 tools/pmc_table.py $O/c${C}_p1 > $O/sq_c$C.txt
  python3 tools/kt_stats.py $O/c${C}_p1 > $O/kt_c$C.txt 2>&1 || true
  cat $O/sq_c$C.txt | head -60
  cat $O/kt_c$C.txt | head -20
done
