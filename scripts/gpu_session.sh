#!/bin/bash
# GPU session stages, comma-separated (default all = tests,bench,prof):
#   tests  pytest -m gpu ($TESTS) + smoke
#   bench  the default bench line (config 3, extra.configs cfg2 / cfg4)
#   prof   rocprofv3 kernel stats of the config-3 bench
#   host   scripts/host_turnaround.py (host share of a scan)
#   pmc    HBM bytes by PMC: config 3 and its dense-map variant
#   vmm    scripts/vmm_probe (growing a reserved range chunk by chunk)
#   dltl   kernel timeline of the drop-in iterate() (scripts/dropin_probe.py under rocprofv3)
# Stops at the first failing step; each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES=${1:-all}
TESTS=${TESTS:-tests}
has() { [[ ",$STAGES," == *",$1,"* || ( $STAGES == all && $1 != host && $1 != pmc && $1 != vmm && $1 != dltl ) ]]; }
if has vmm; then
  timeout -k 10 120 ./scripts/vmm_probe > gpurun_out/vmm_probe.txt 2>&1 || { echo vmm probe failed; tail -20 gpurun_out/vmm_probe.txt; exit 8; }
  tail -1 gpurun_out/vmm_probe.txt
fi
if has tests; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -rf --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
  if [[ $rc -ne 0 ]]; then exit 10; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
  tail -1 gpurun_out/smoke.log
fi
if has host; then
  timeout -k 10 300 python scripts/host_turnaround.py > gpurun_out/host_turnaround.json 2> gpurun_out/host_turnaround.err || { echo host failed; tail -20 gpurun_out/host_turnaround.err; exit 6; }
  cut -c1-600 gpurun_out/host_turnaround.json
fi
if has bench; then
  timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 4; }
  tail -1 gpurun_out/bench.log | cut -c1-400
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python bench.py --no-cpu-baseline --no-extras > gpurun_out/prof.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof.log; exit 5; }
  python scripts/prof_summary.py /tmp/prof gpurun_out/prof_summary.txt "${PROF_TITLE:-}" > /dev/null && head -14 gpurun_out/prof_summary.txt
  python3 scripts/timeline.py "$(find /tmp/prof -name '*.db' | sort | tail -n 1)" 23 > gpurun_out/bench_timeline.txt || echo "(no timeline)"
fi
if has dltl; then
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/dl -o dl -- python3 scripts/dropin_probe.py > gpurun_out/dropin_probe.log 2>&1 || { echo dropin trace failed; tail -20 gpurun_out/dropin_probe.log; exit 9; }
  python3 scripts/timeline.py "$(find /tmp/dl -name '*.db' | sort | tail -n 1)" 3 > gpurun_out/dropin_timeline.txt && grep -v "^W20\|^E20" gpurun_out/dropin_probe.log | tail -2
fi
if has pmc; then
  PMC_OUT=gpurun_out/pmc3 bash scripts/pmc_round.sh || { echo pmc failed; exit 7; }
  BENCH_ARGS="--no-cpu-baseline --no-extras --map dense" PMC_OUT=gpurun_out/pmcd bash scripts/pmc_round.sh || { echo pmc dense failed; exit 7; }
  echo pmc done
fi
