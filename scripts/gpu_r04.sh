#!/bin/bash
# Round-4 GPU session stages: tests (+ smoke), bench (config 3 line with the
# config 2 / 4 lines in extra.configs), prof (rocprofv3 kernel stats of the
# config-3 bench).  Stops at the first failing step; each GPU step has its own
# time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
TESTS=${TESTS:-tests}
if [[ $STAGE == all || $STAGE == tests ]]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -rf --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  if [[ $rc -ne 0 ]]; then exit 10; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
  tail -1 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 4; }
  tail -1 gpurun_out/bench.log | cut -c1-400
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python bench.py --no-cpu-baseline --no-extras > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof.log; exit 5; }
  python scripts/prof_summary.py /tmp/prof gpurun_out/prof_summary.txt "${PROF_TITLE:-}" > /dev/null && head -14 gpurun_out/prof_summary.txt
fi
