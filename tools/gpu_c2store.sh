#!/bin/bash
# Config 2: is the output store behind the ring kernel's fetch above its loads?
# A/B of the default kernel, no-store (a14) and loads-only (a3), then one
# FETCH_SIZE / WRITE_SIZE pass over the same variants (per-kernel rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROUND:-r02c2s}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip --variants ${VARIANTS:-c2,a14,a3} --rounds 3 > gpurun_out/ab_$R.log 2>&1; step ab $?
tail -1 gpurun_out/ab_$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d.get('variants_ab'))"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${R}_$C -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling --variants ${VARIANTS:-c2,a14,a3} --rounds 1 > gpurun_out/pmc_${R}_$C.log 2>&1; step pmc_$C $?
done
python3 tools/pmc_summary.py gpurun_out/pmc_${R}_FETCH_SIZE gpurun_out/pmc_${R}_WRITE_SIZE config2 > gpurun_out/pmc_summary_$R.json
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_summary_$R.json'))
for k,v in d['config2']['kernels'].items(): print(k[:48], v['dispatches'], v['fetch_bytes_corrected']/1e9, v['write_bytes']/1e9)"
