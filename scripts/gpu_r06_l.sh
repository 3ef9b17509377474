#!/bin/bash
# round 6 (second session): the overflow scan's next row descriptor in flight --
# parity first, then a same-box A/B on the dense map (every list overflows) and the grid
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py > gpurun_out/tests_l.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_l.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 2 --steps 10 --bench-args "--map dense" base=fast-slam_amd/lib/libfs2_base.so \
    pf=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_l_dense.json > gpurun_out/ab_l_dense.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_l_dense.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_lib.py --rounds 2 base=fast-slam_amd/lib/libfs2_base.so \
    pf=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_l_grid.json > gpurun_out/ab_l_grid.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_l_grid.log
exit $rc
