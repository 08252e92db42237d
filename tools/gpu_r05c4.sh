#!/bin/bash
# round 5: per-wave guess / walk clock of the four-lane segment walk (clock build C4), 2 MiB and 1 MiB segments
set -o pipefail
O=gpurun_out/${OUT:-r05c4}; mkdir -p $O
L=lsm_storage_engine_amd
cp $L/liblsmck.so /tmp/liblsmck_keep.so
cp $L/ab/C4.so $L/liblsmck.so
for S in ${SIZES:-0 1048576}; do
  SEG_CLOCK_LANES=${LANES:-4} SEG_CLOCK_SEG_BYTES=$S timeout -k 10 300 python3 -u tools/seg_clock.py > $O/clock_$S.log 2>&1 || { echo "clock $S failed"; tail -5 $O/clock_$S.log; cp /tmp/liblsmck_keep.so $L/liblsmck.so; exit 1; }
  tail -n 1 $O/clock_$S.log
done
cp /tmp/liblsmck_keep.so $L/liblsmck.so
