#!/bin/bash
# WAL walk part size: the WAL GPU tests, the full-size config-3w replay test,
# then the full-size device replay rate (tools/wal_replay_big.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r03v}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wal.py "tests/test_gpu_crc.py::test_config3w_full_size_summary" -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/pytest_wal_$R.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_wal_$R.log; [ $rc -eq 0 ] || exit $rc
LSMCK_WAL_TRACE=1 timeout -k 10 400 python3 tools/wal_replay_big.py --steps 3 > gpurun_out/wal_replay_big_$R.json 2> gpurun_out/wal_replay_big_$R.log; rc=$?
grep -c "mark+scan" gpurun_out/wal_replay_big_$R.log; grep "replay\|crc+compare" gpurun_out/wal_replay_big_$R.log | tail -5; cat gpurun_out/wal_replay_big_$R.json
exit $rc
