cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02b.log 2>&1; echo "smoke rc=$?"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02b.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_r02b.log; echo "pytest rc=$rc"
