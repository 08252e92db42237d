#!/bin/bash
# Stream-kernel change check: its GPU tests and the config-3 full-size digest,
# an interleaved A/B of variants on config 3, and one FETCH_SIZE / WRITE_SIZE
# pass of the default config-3 bench.  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02q}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_stream.py "tests/test_gpu_crc.py::test_config3_full_size_summary" ${EXTRA_TESTS} -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_$R.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_$R.log; step pytest $rc
timeout -k 10 400 python3 bench.py --config ${CFG:-3} --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip --variants ${VARIANTS:-c0,c0t0,a3} --rounds 3 > gpurun_out/ab_$R.log 2>&1; step ab $?
tail -1 gpurun_out/ab_$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline'], d.get('variants_ab'))"
[ -n "$SKIP_PMC" ] && exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_$C -o pmc -- python3 bench.py --config ${CFG:-3} --steps 3 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/pmc_${R}_$C.log 2>&1; step pmc_$C $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_${R}_FETCH_SIZE gpurun_out/pmc_${R}_WRITE_SIZE config${CFG:-3} > gpurun_out/pmc_summary_$R.json
cat gpurun_out/pmc_summary_$R.json
