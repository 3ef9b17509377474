#!/bin/bash
# round 6: (1) FS2_GUARD catches the round-5 np_part overrun (variant with the old
# size: the guard test must FAIL naming h->np_part); (2) A/B: k_update without
# the motion sample (timing only) vs the product build
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FS2_LIB=$PWD/fast-slam_amd/lib/libfs2_oldnp.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 \
    --timeout-method thread tests/test_gpu_guards.py -k "1000000" > gpurun_out/guard_validate.log 2>&1
rc=$?
echo "guard validation rc=$rc (1 expected: the overrun is found)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u scripts/ab_lib.py --rounds 3 movecand=fast-slam_amd/lib/libfs2.so \
    moveupd=fast-slam_amd/lib/libfs2_moveupd.so nomove=fast-slam_amd/lib/libfs2_nomove.so \
    --out gpurun_out/ab_nomove.json > gpurun_out/ab_nomove.log 2>&1
rc=$?
cat gpurun_out/ab_nomove.log | grep '^{'
grep -E "guard bytes|passed|failed" gpurun_out/guard_validate.log | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mtrng.py \
    tests/test_gpu_dropin.py tests/test_gpu_pipelined.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py \
    tests/test_gpu_exact.py > gpurun_out/tests_c.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_c.log
exit $rc
