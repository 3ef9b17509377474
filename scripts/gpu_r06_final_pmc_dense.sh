#!/bin/bash
# round 6 final build: PMC passes of the dense-map variant (bench.py --map dense)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BENCH_ARGS="--no-cpu-baseline --no-extras --map dense" PMC_OUT=gpurun_out/pmc_dense_v6 bash scripts/pmc_round.sh || { echo pmc failed; exit 5; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --map dense > gpurun_out/dense_v6.log 2>&1 || { echo bench failed; tail -20 gpurun_out/dense_v6.log; exit 4; }
ls gpurun_out/pmc_dense_v6
