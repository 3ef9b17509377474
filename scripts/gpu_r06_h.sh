#!/bin/bash
# round 6 (second session): exact fmod fast path + shared post-EKF inverse in
# k_update; double-buffered page copies as a variant -- parity first, then a
# same-box A/B against HEAD's build; timing-only probes of the candidate pass (half the page loads; 8-byte loads)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_gpu_exact.py > gpurun_out/tests_h.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_h.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/ab_lib.py --rounds 2 base=fast-slam_amd/lib/libfs2_base.so \
    new=fast-slam_amd/lib/libfs2.so b1db=fast-slam_amd/lib/libfs2_b1db.so half=fast-slam_amd/lib/libfs2_half.so x2=fast-slam_amd/lib/libfs2_x2.so --out gpurun_out/ab_h.json > gpurun_out/ab_h.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_h.log
exit $rc
