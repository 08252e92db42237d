#!/bin/bash
# Probe: the segment walk on large device-resident logs, phases traced (LSMCK_WAL_TRACE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R:-r04c}
mkdir -p $O
for N in 1048576 4194304 16777216 67108864; do
  echo "== records $N" >&2
  LSMCK_WAL_TRACE=1 timeout -k 10 150 python3 -u tools/wal_replay_big.py --steps 2 --records $N > $O/walprobe_$N.log 2>&1
  rc=$?
  echo "== rc=$rc" >&2
  tail -4 $O/walprobe_$N.log >&2
  [ $rc -eq 0 ] || exit $rc
done
