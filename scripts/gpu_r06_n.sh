#!/bin/bash
# round 6 (second session), 4-byte descriptors: PMC passes (HBM bytes of the
# update kernels and the gather), then a kernel trace of the headline bench with
# its stats summary and the scan timeline
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_OUT=gpurun_out/pmc_v5 bash scripts/pmc_round.sh || { echo pmc failed; exit 5; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v5 -o run -- python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/prof_v5.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_v5.log; exit 6; }
python3 scripts/prof_summary.py gpurun_out/prof_v5 gpurun_out/prof_v5_summary.txt "r06-v5 (4-byte descriptors): python bench.py --no-cpu-baseline --no-extras" > /dev/null && head -30 gpurun_out/prof_v5_summary.txt
db=$(python3 -c "import glob; print((glob.glob('gpurun_out/prof_v5/**/*.db', recursive=True) + [''])[0])")
[ -n "$db" ] && python3 scripts/timeline.py "$db" 23 > gpurun_out/timeline_v5.txt
find gpurun_out/prof_v5 -name '*.db' -delete
tail -1 gpurun_out/prof_v5.log
