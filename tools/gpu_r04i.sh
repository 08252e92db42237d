#!/bin/bash
# WAL session: the GPU WAL tests (segment walk, device records, prefix code),
# the small and the 97.8 GiB replays with records to host and on the device,
# segment-size sweeps, kernel traces of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R:-r04i}
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
step pytest_wal 400 python3 -u -m pytest tests/test_gpu_wal.py -q -x --timeout 200 --timeout-method thread
step small 150 env WAL_KT_SEGS=512,1024,2048,4096,16384 python3 -u tools/wal_kt.py
step big 400 env LSMCK_WAL_TRACE=1 python3 -u tools/wal_replay_big.py --steps 3 --device-recs 1 --seg-sweep 65536,262144,1048576,4194304
step kt_small 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_small -o kt -- python3 tools/wal_kt.py
python3 tools/kt_stats.py $O/kt_small > $O/kt_stats_small.txt 2>&1
step kt_big 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_big -o kt -- python3 tools/wal_replay_big.py --steps 2 --device-recs 1
python3 tools/kt_stats.py $O/kt_big > $O/kt_stats_big.txt 2>&1
echo "== done" >&2
