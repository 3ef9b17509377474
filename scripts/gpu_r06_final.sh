#!/bin/bash
# round 6 final build: the whole GPU suite, smoke, the default bench line, and a
# kernel trace with its stats summary and the scan timeline
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/final_tests.log 2>&1
rc=$?
tail -n 3 gpurun_out/final_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/final_smoke.log; exit 3; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final_bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/final_bench.log; exit 4; }
tail -1 gpurun_out/final_bench.log | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v6 -o run -- python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/prof_v6.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_v6.log; exit 6; }
python3 scripts/prof_summary.py gpurun_out/prof_v6 gpurun_out/prof_v6_summary.txt "r06-v6 final build: python bench.py --no-cpu-baseline --no-extras" > /dev/null && head -32 gpurun_out/prof_v6_summary.txt
db=$(python3 -c "import glob; print((glob.glob('gpurun_out/prof_v6/**/*.db', recursive=True) + [''])[0])")
[ -n "$db" ] && python3 scripts/timeline.py "$db" 23 > gpurun_out/timeline_v6.txt
find gpurun_out/prof_v6 -name '*.db' -delete
tail -1 gpurun_out/prof_v6.log | cut -c1-300
