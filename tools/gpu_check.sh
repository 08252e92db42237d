#!/bin/bash
# One GPU call: smoke, GPU parity tests, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; a crash (rc > 1 from pytest, or any
# non-zero from the others) ends the script before the next GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r01}
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf --timeout 600 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 300 python3 bench.py ${BENCH_ARGS} > gpurun_out/bench_$R.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_$R.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$R -o bench -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_$R.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_$R.log
find gpurun_out/prof_$R -name "*stats*" | head
