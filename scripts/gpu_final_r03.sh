#!/bin/bash
# Round-3 final GPU session: GPU tests + smoke, config-3 bench, rocprof kernel
# stats, PMC passes (scripts/pmc_round.sh), config-4 and config-2 bench lines.
# Stops at the first failing step; every GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_r03.sh tests || exit $?
bash scripts/gpu_r03.sh bench || exit $?
PROF_TITLE="${PROF_TITLE:-r03 final}" bash scripts/gpu_r03.sh prof || exit $?
bash scripts/pmc_round.sh || { echo "pmc failed"; exit 6; }
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline --no-extras > gpurun_out/bench_cfg4.log 2>&1 || { echo "cfg4 bench failed"; tail -20 gpurun_out/bench_cfg4.log; exit 7; }
timeout -k 10 300 python bench.py --config 2 --no-cpu-baseline --no-extras > gpurun_out/bench_cfg2.log 2>&1 || { echo "cfg2 bench failed"; tail -20 gpurun_out/bench_cfg2.log; exit 8; }
tail -1 gpurun_out/bench_cfg4.log | cut -c1-300
tail -1 gpurun_out/bench_cfg2.log | cut -c1-300
