set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04a/pytest_wal.log 2>&1 || { tail -30 gpurun_out/r04a/pytest_wal.log; exit 1; }
tail -3 gpurun_out/r04a/pytest_wal.log
LSMCK_WAL_TRACE=1 timeout -k 10 300 python -u tools/wal_replay_big.py --steps 3 > gpurun_out/r04a/big.json 2> gpurun_out/r04a/big.err || { tail -20 gpurun_out/r04a/big.err; exit 1; }
cat gpurun_out/r04a/big.json
timeout -k 10 200 python -u tools/wal_diag.py > gpurun_out/r04a/diag.json 2> gpurun_out/r04a/diag.err || { tail -20 gpurun_out/r04a/diag.err; exit 1; }
cat gpurun_out/r04a/diag.json
