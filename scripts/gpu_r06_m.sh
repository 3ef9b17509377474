#!/bin/bash
# round 6 (second session): 4-byte page descriptors (page id only; boxes per
# workgroup row) -- the whole GPU suite first, then same-box A/B on the headline
# grid and on the dense map
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/tests_m.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_m.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 3 base=fast-slam_amd/lib/libfs2_base.so \
    desc4=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_m_grid.json > gpurun_out/ab_m_grid.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_m_grid.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/ab_lib.py --rounds 1 --steps 10 --bench-args "--map dense" base=fast-slam_amd/lib/libfs2_base.so \
    desc4=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_m_dense.json > gpurun_out/ab_m_dense.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_m_dense.log
exit $rc
