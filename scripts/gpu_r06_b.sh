#!/bin/bash
# round 6: buffer-end guards first (the N = 8e6 fault), then the appended-maps
# parity test, the N = 8e6 drift history (guarded), and the sharded tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_guards.py \
    > gpurun_out/tests_guards.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_appended.py \
    > gpurun_out/tests_appended.log 2>&1 &&
timeout -k 10 400 python -u scripts/drift_study.py dump --particles 8000000 --landmarks 100 --scans 30 --guard \
    --out gpurun_out/drift_N8e6_L100.npz > gpurun_out/drift_8e6.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_sharded_procs.py tests/test_gpu_pool_growth.py tests/test_gpu_config5_shape.py \
    > gpurun_out/tests_a.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_guards.log gpurun_out/tests_appended.log gpurun_out/drift_8e6.log gpurun_out/tests_a.log 2>/dev/null
exit $rc
