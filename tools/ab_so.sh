cd $GRAFT_REPO_ROOT
L=lsm_storage_engine_amd
run() { timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/ab_$1_c2.log 2>&1 && timeout -k 10 200 python -u bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-roundtrip --no-stream-ceiling > gpurun_out/ab_$1_c3.log 2>&1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_crc.py tests/test_gpu_wal.py > gpurun_out/crc_tests_new.log 2>&1 || exit 1
run new1 || exit 1
cp $L/liblsmck_head.so $L/liblsmck.so && run old || exit 1
cp $L/liblsmck_new.so $L/liblsmck.so && run new2 || exit 1
