#!/bin/bash
# Config 2 output-store A/B: ring tile orders (strided, contiguous + queued
# 256-B blocks, strided + LDS-gathered), no-store ablations, with parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_async.py::test_fixed_ring_tile_orders" -x -q -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_${ROUND:-r02c2q}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${ROUND:-r02c2q}.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-c2,a14,c2o3,c2o4,a14o1,a3} ROUND=${ROUND:-r02c2q} bash tools/gpu_c2store.sh
