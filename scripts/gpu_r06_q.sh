#!/bin/bash
# round 6 (second session): the candidate pass's descriptor prefetch depth
# (2 vs 4; 4-byte descriptors) on the 32-row gather tiles -- same-box A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/ab_lib.py --rounds 3 da2=fast-slam_amd/lib/libfs2.so \
    da4=fast-slam_amd/lib/libfs2_da4.so --out gpurun_out/ab_q.json > gpurun_out/ab_q.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_q.log
exit $rc
