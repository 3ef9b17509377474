#!/bin/bash
# round 6: summary grid fitted to the extent (not a power of two) -- parity first,
# then a same-box A/B against the power-of-two grid and the round-5 motion placement
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_sharded.py tests/test_gpu_guards.py \
    tests/test_gpu_appended.py > gpurun_out/tests_f.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_f.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/ab_lib.py --rounds 3 fit=fast-slam_amd/lib/libfs2.so \
    pow2=fast-slam_amd/lib/libfs2_pow2.so --out gpurun_out/ab_cell.json > gpurun_out/ab_cell.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_cell.log
exit $rc
