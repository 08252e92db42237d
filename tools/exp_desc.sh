cd $GRAFT_REPO_ROOT
run() { # name args...
  n=$1; shift
  timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --rounds 3 "$@" > gpurun_out/x_$n.log 2>&1 || return 1
  tail -1 gpurun_out/x_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],2), {k:round(v['median_ms'],2) for k,v in d.get('variants_ab',{}).items()})"
}
timeout -k 10 100 ./tools/microbench_loads 64 2>&1 | head -1
run c2fixed --config 2 --variants c1,c2,a3 &&
run c2desc --config 2 --desc --variants c1,c2,a3 &&
run c3a16 --config 3 --pack-align 16 --variants c1,a3 &&
run c3a128 --config 3 --pack-align 128 --variants c1,a3 &&
run c3 --config 3 --variants c1,a3
