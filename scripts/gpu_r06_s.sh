#!/bin/bash
# round 6 (second session): the gather's row-tile workgroups first (1024 of them,
# beside the per-output blocks) and / or the next tile's source load in flight --
# same-box A/B against the final build
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/ab_lib.py --rounds 2 cur=fast-slam_amd/lib/libfs2_cur.so \
    tf=fast-slam_amd/lib/libfs2_tf.so tfp=fast-slam_amd/lib/libfs2_tfp.so pipe=fast-slam_amd/lib/libfs2_pipe.so \
    --out gpurun_out/ab_s.json > gpurun_out/ab_s.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_s.log
exit $rc
