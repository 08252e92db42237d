cd $GRAFT_REPO_ROOT
run() { # name args...
  n=$1; shift
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-roundtrip --rounds 3 "$@" > gpurun_out/x_$n.log 2>&1 || return 1
  tail -1 gpurun_out/x_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],2), {k:round(v['median_ms'],2) for k,v in d.get('variants_ab',{}).items()})"
}
timeout -k 10 100 ./tools/microbench_loads 64 2>&1 | head -1
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_x.log 2>&1; tail -3 gpurun_out/pytest_x.log
run c2 --config 2 --variants c1,c2,c4,g2,a1,a3,a2 &&
run c3 --config 3 --variants c1,c2,c4,a1,a3,a2
