cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/wt.so
for N in A L; do
  cp $L/ab/$N.so $L/liblsmck.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04v/kt_$N -o kt -- python3 tools/wal_replay_big.py --steps 2 --device-recs 1 > gpurun_out/r04v/kt_$N.log 2>&1 || { cp /tmp/wt.so $L/liblsmck.so; exit 1; }
  python3 tools/kt_stats.py gpurun_out/r04v/kt_$N > gpurun_out/r04v/kt_stats_$N.txt 2>&1
  grep -E "seg_walk |seg_repair|seg_place" gpurun_out/r04v/kt_stats_$N.txt
done
cp /tmp/wt.so $L/liblsmck.so
