#!/bin/bash
# round 6 (second session): the gather's row tiles, 8 / 16 / 32 rows high --
# same-box A/B on the headline (tail_ms holds the gather)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/ab_lib.py --rounds 3 t8=fast-slam_amd/lib/libfs2.so \
    t16=fast-slam_amd/lib/libfs2_t16.so t32=fast-slam_amd/lib/libfs2_t32.so --out gpurun_out/ab_p.json > gpurun_out/ab_p.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_p.log
exit $rc
