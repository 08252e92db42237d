#!/bin/bash
# Round 4, first GPU session: the segment walk (WAL tests, the 97.8 GiB and
# 0.24 GB replays, their kernel traces), the N-rank bench rehearsal, the
# default bench line, the server's compaction tick, the SHA-256 sorted
# descriptors A/B.  Each step has its own time limit; a test failure goes on
# to the next step, a timeout / abort / crash ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -3 $O/$name.log >&2
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "== stopping after $name (rc $rc)" >&2
    exit $rc
  fi
  return 0
}
O=gpurun_out/${R:-r04a}
mkdir -p $O
step pytest_wal 500 python -u -m pytest tests/test_gpu_wal.py -v --timeout 200 --timeout-method thread
step pytest_stream 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_crc.py -x -v --timeout 300 --timeout-method thread
step wal_big 300 env LSMCK_WAL_TRACE=1 python -u tools/wal_replay_big.py --steps 3
step wal_diag 240 python -u tools/wal_diag.py
step pytest_bench 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread
step bench_default 300 python -u bench.py
step pytest_server 400 python -u -m pytest tests/test_server.py -v --timeout 300 --timeout-method thread
step sha_ab 300 python -u bench.py --digest sha256 --variants=-,d1 --rounds 3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip --no-config4
step pytest_sha 400 python -u -m pytest tests/test_gpu_sha.py -x -v --timeout 200 --timeout-method thread -k "short_tail or length_sorted"
step kt_wal_big 300 rocprofv3 --kernel-trace --stats -d $O/kt_wal_big -o run -- python3 tools/wal_replay_big.py --steps 2
echo done >&2
