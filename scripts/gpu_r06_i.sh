#!/bin/bash
# round 6 (second session): k_update phase breakdown of the current build
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FS2_LIB=fast-slam_amd/lib/libfs2_timing.so timeout -k 10 300 python3 -u scripts/phase_timing.py > gpurun_out/phase_i.txt 2>&1
rc=$?
cat gpurun_out/phase_i.txt
exit $rc
