#!/bin/bash
# Probe: the segment walk on large device-resident logs, phases traced (LSMCK_WAL_TRACE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R:-r04c}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wal.py -q -x --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1 || { tail -5 $O/pytest_wal.log >&2; exit 1; }
tail -2 $O/pytest_wal.log >&2
for N in 1048576 4194304 16777216 67108864; do
  echo "== records $N" >&2
  LSMCK_WAL_TRACE=1 timeout -k 10 150 python3 -u tools/wal_replay_big.py --steps 2 --records $N > $O/walprobe_$N.log 2>&1
  rc=$?
  echo "== rc=$rc" >&2
  tail -4 $O/walprobe_$N.log >&2
  [ $rc -eq 0 ] || exit $rc
done
