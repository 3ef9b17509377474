#!/bin/bash
# round 6 (second session): phase B's descriptors and reserved pages staged in LDS
# during phase A -- parity first, then a same-box A/B against HEAD's build
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_exact.py tests/test_gpu_appended.py tests/test_gpu_sharded.py > gpurun_out/tests_j.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_j.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u scripts/ab_lib.py --rounds 3 base=fast-slam_amd/lib/libfs2_base.so \
    staged=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_j.json > gpurun_out/ab_j.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_j.log
exit $rc
