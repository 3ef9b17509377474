#!/bin/bash
# round 6 (second session): page-table rows copied in row-major tiles (gather_rows) on top of the 4-byte
# descriptors -- the whole GPU suite first, then same-box A/B on the headline
# grid, and a kernel trace (the gather's time)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/tests_o.log 2>&1
rc=$?
tail -n 3 gpurun_out/tests_o.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab_lib.py --rounds 3 desc4=fast-slam_amd/lib/libfs2_desc4.so \
    tiles=fast-slam_amd/lib/libfs2.so --out gpurun_out/ab_o_grid.json > gpurun_out/ab_o_grid.log 2>&1
rc=$?
grep '^{' gpurun_out/ab_o_grid.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_o -o run -- python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/prof_o.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_o.log; exit 6; }
db=$(python3 -c "import glob; print((glob.glob('gpurun_out/prof_o/**/*.db', recursive=True) + [''])[0])")
[ -n "$db" ] && python3 scripts/timeline.py "$db" 23 > gpurun_out/timeline_o.txt
find gpurun_out/prof_o -name '*.db' -delete
grep k_gather gpurun_out/timeline_o.txt | awk '$3 > 20'
