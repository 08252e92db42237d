#!/bin/bash
# round 5: where config 3's stream kernel is bound -- SQ counters and the
# effective clock (GRBM_GUI_ACTIVE / 8 / wall, MI355X_MICROARCH.md "DVFS")
# of the full kernel and its ablations (a5: every tile on the no-event path,
# with loads; a3: payload loads only; a2: compute only), one build with the
# ablations compiled in (tools/build_ab.sh SQ WT), plus their same-process times.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05sq; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_wt.so
cp $L/ab/SQ.so $L/liblsmck.so
B="python3 bench.py --config 3 --steps 3 --warmup 1 --rounds 1 --variants=-,a5,a3,a2 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4"
timeout -k 10 200 python3 bench.py --config 3 --steps 5 --warmup 2 --rounds 5 --variants=-,a5,a3,a2 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4 > $O/times.log 2>&1 || { echo times failed; tail -5 $O/times.log; cp /tmp/liblsmck_wt.so $L/liblsmck.so; exit 1; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_WAVES GRBM_COUNT"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/p$n -o p -- $B > $O/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/p$n.log; cp /tmp/liblsmck_wt.so $L/liblsmck.so; exit 1; }
done
cp /tmp/liblsmck_wt.so $L/liblsmck.so
python3 tools/pmc_table.py $O/p1 $O/p2 > $O/sq_table.txt 2>&1
tail -n 1 $O/times.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get("variants_ab")))'
cat $O/sq_table.txt | head -80
