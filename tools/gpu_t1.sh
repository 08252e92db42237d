cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_async.py tests/test_gpu_wal.py tests/test_tree.py tests/test_gpu_bench.py tests/test_abi.py > gpurun_out/t1.log 2>&1
rc=$?; tail -30 gpurun_out/t1.log; exit $rc
