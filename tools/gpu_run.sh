#!/bin/bash
# The one GPU-box runner (replaces the per-session tools/gpu_r0*.sh scripts,
# which stay in git history up to d60fa90).  Run as
#   gpurun -- 'ROUND=r06a STEPS="smoke tests" TESTS=tests/test_gpu_wal_lengths.py bash tools/gpu_run.sh'
# Steps picked by STEPS (space list), run in this order:
#   build smoke tests pytest bench benchkt c3pmc walbig walbigkt walmib wallogs waldiag sha shaab tree server
#   custom (runs $CUSTOM under the same time limit / stop rules)
# Logs go to gpurun_out/$ROUND/<step>.log.  A test failure goes on to the next
# step; a timeout / abort / crash (rc 124, 137, 134, 139, > 128) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r06}
O=gpurun_out/$R
mkdir -p $O
STEPS=${STEPS:-"smoke pytest bench benchkt"}
has() { [[ " $STEPS " == *" $1 "* ]]; }
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
has smoke && step smoke 240 python3 -c "import __graft_entry__ as g; g.smoke()"
# a chosen subset of the GPU tests (TESTS: pytest targets; PYTEST_K: a -k expression)
has tests && step tests ${TESTS_SECS:-600} python3 -u -m pytest ${TESTS:-tests} -m gpu -v -rf --timeout 300 \
  --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
has pytest && step pytest 1100 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
# the driver's default line, then the same command (no host round trip: its
# staged host batches run the stream kernel too) under the kernel trace, so the
# line's HIP-event launch time and the trace's durations come from the same launches
has bench && step bench 400 python3 bench.py
if has benchkt; then
  step benchkt 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c3 -o kt -- python3 bench.py --no-host-roundtrip
  python3 tools/kt_stats.py $O/kt_c3 > $O/kt_stats_c3.txt 2>&1
fi
if has c3pmc; then  # HBM bytes per launch of the stream kernel (separate FETCH_SIZE / WRITE_SIZE passes)
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc_c3_$C 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_c3_$C -o pmc -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --no-config4
  done
  python3 tools/pmc_summary.py $O/pmc_c3_FETCH_SIZE $O/pmc_c3_WRITE_SIZE config3 > $O/pmc_summary_c3.json 2>&1
fi
# the 97.8 GiB config-3w log: compact records to a pinned host array (SDMA read-back) and in HBM
has walbig && step walbig 300 env LSMCK_WAL_TRACE=1 python3 -u tools/wal_replay_big.py --steps 5 --compact 1 --device-recs 1 ${WALBIG_ARGS}
if has walbigkt; then
  step walbigkt 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_walbig -o kt -- python3 tools/wal_replay_big.py --steps 2 --compact 1 --device-recs 1 ${WALBIG_ARGS}
  python3 tools/kt_stats.py $O/kt_walbig > $O/kt_stats_walbig.txt 2>&1
fi
has walmib && step walmib 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape mib
has wallogs && step wallogs 300 python3 -u tools/wal_replay_big.py --steps 3 --compact 1 --device-recs 1 --shape logs
if has waldiag; then
  step waldiag 300 python3 -u tools/wal_diag.py
  step waldiagkt 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_waldev -o kt -- python3 tools/wal_kt.py
  python3 tools/kt_stats.py $O/kt_waldev > $O/kt_stats_waldev.txt 2>&1
fi
has sha && step sha 400 python3 bench.py --digest sha256 --steps 5 --warmup 1 --no-config4
has shaab && step shaab 600 python3 bench.py --digest sha256 --variants=${SHA_VARIANTS:--,t6,t16} --rounds 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-config4
has tree && step tree 900 python3 -u tools/e2e_tree.py --gib 16 --reps 2 --multi 2 --dir /dev/shm/lsm_e2e_$R
has server && step server 1100 python3 -u tools/e2e_server.py --gib 100 --dir /dev/shm/lsm_e2e_server_$R
has custom && step custom ${CUSTOM_SECS:-300} bash -c "$CUSTOM"
echo "== done" >&2
