#!/bin/bash
# Round-3 GPU session: the given pytest selection, smoke, bench, kernel trace.
#   scripts/gpu_r03.sh [tests|bench|prof|all] [pytest args...]
# Every GPU step has its own time limit; the script stops at the first failure
# other than pytest's "tests failed" (1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
shift || true
if [[ $STAGE == all || $STAGE == tests ]]; then
  SEL=("$@")
  [[ ${#SEL[@]} -eq 0 ]] && SEL=(tests -m gpu)
  timeout -k 10 900 python -u -m pytest "${SEL[@]}" -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests.log
  if [[ $rc -ne 0 ]]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
  tail -1 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 4; }
  tail -1 gpurun_out/bench.log | cut -c1-1500
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  rm -rf /tmp/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python bench.py --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof.log; exit 5; }
  python scripts/prof_summary.py /tmp/prof gpurun_out/prof_summary.txt "${PROF_TITLE:-}" > /dev/null && head -30 gpurun_out/prof_summary.txt
  db=$(find /tmp/prof -name "*.db" | head -1)
  if [[ -n "$db" ]]; then python scripts/timeline.py "$db" 4 > gpurun_out/timeline.txt; cp "$db" gpurun_out/run.db; fi
fi
