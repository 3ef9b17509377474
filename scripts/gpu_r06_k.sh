#!/bin/bash
# round 6 (second session): the overflow scan only for the measurements with
# candidates past an overflowing list -- parity first, then same-box A/B on the
# dense map (where every list overflows) and on the headline grid
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_appended.py > gpurun_out/tests_k.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_k.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 2 --steps 10 --bench-args "--map dense" base=fast-slam_amd/lib/libfs2_base.so \
    ovm=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_k_dense.json > gpurun_out/ab_k_dense.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_k_dense.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_lib.py --rounds 2 base=fast-slam_amd/lib/libfs2_base.so \
    ovm=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_k_grid.json > gpurun_out/ab_k_grid.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_k_grid.log
exit $rc
