#!/bin/bash
# round 6: same-box A/B of the session-start build (0ab01c6) against the final one
# on the headline (3 rounds) and the dense map (1 round)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/ab_lib.py --rounds 3 start=fast-slam_amd/lib/libfs2_start.so \
    final=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_r_grid.json > gpurun_out/ab_r_grid.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_r_grid.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_lib.py --rounds 1 --steps 10 --bench-args "--map dense" start=fast-slam_amd/lib/libfs2_start.so \
    final=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_r_dense.json > gpurun_out/ab_r_dense.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_r_dense.log
exit $rc
