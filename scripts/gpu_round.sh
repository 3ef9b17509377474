#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first crash/timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
python -c "import torch; print('torch', torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))" > gpurun_out/env.log 2>&1
if [[ $STAGE == all || $STAGE == tests ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
  tail -1 gpurun_out/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 4; }
  tail -1 gpurun_out/bench.log
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python bench.py --no-cpu-baseline --no-extras > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof.log; exit 5; }
  python scripts/prof_summary.py /tmp/prof gpurun_out/prof_summary.txt "${PROF_TITLE:-}" > /dev/null && head -12 gpurun_out/prof_summary.txt
fi
