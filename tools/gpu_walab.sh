#!/bin/bash
# Same-box A/B of library builds (tools/build_ab.sh) on the device WAL replay:
# the 0.24 GB wal_diag image (tools/wal_kt.py) and a framed config-3 log of
# $BIG records (tools/wal_replay_big.py), each build in turn, $ROUNDS rounds.
#   LIBS="A B" ROUNDS=2 BIG=16777216 R=r04g bash tools/gpu_walab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export WAL_KT_DEVRECS=${WAL_KT_DEVRECS:-0}  # (builds before LSMCK_RECS_DEVICE would misread the flag)
O=gpurun_out/${R:-walab}
mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_wt.so
restore() { cp /tmp/liblsmck_wt.so $L/liblsmck.so; }
for r in $(seq 1 ${ROUNDS:-2}); do
  for N in $LIBS; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 150 python3 -u tools/wal_kt.py > $O/small_${N}_$r.log 2>&1 || { echo "small $N failed rc=$?"; tail -5 $O/small_${N}_$r.log; restore; exit 1; }
    echo "$N round $r small: $(tail -1 $O/small_${N}_$r.log)"
    timeout -k 10 300 python3 -u tools/wal_replay_big.py --steps 3 --records ${BIG:-16777216} $BIG_ARGS > $O/big_${N}_$r.log 2>&1 || { echo "big $N failed rc=$?"; tail -5 $O/big_${N}_$r.log; restore; exit 1; }
    echo "$N round $r big: $(tail -1 $O/big_${N}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_median"], d["value"], d["summary_matches_oracle"], d["seg_repairs"], d.get("records_on_device"))')"
  done
done
restore
# then, with KT=1, a kernel trace of the small replay per build
if [ -n "$KT" ]; then
  for N in $LIBS; do
    cp $L/ab/$N.so $L/liblsmck.so
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_small_$N -o kt -- python3 tools/wal_kt.py > $O/kt_small_$N.log 2>&1 || { echo "kt $N failed"; restore; exit 1; }
    python3 tools/kt_stats.py $O/kt_small_$N > $O/kt_stats_small_$N.txt 2>&1
    grep -E "wal_seg|crc32_stream|copyBuffer" $O/kt_stats_small_$N.txt | head -8
  done
  restore
fi
