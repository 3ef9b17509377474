#!/bin/bash
# round 6: drift histories for the shard-policy study + the sharded tests touched by the ADVICE fixes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/drift_study.py dump --particles 1000000 --landmarks 500 --scans 30 \
    --out gpurun_out/drift_N1e6_L500.npz > gpurun_out/drift_1e6.log 2>&1 &&
timeout -k 10 300 python -u scripts/drift_study.py dump --particles 8000000 --landmarks 100 --scans 30 \
    --out gpurun_out/drift_N8e6_L100.npz > gpurun_out/drift_8e6.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_appended.py tests/test_gpu_sharded_procs.py tests/test_gpu_pool_growth.py tests/test_gpu_config5_shape.py \
    > gpurun_out/tests_a.log 2>&1
rc=$?
tail -5 gpurun_out/tests_a.log
exit $rc
