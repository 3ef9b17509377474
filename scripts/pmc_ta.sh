#!/bin/bash
# Address-path counters of the update kernels (one pass, no traces): TA busy /
# stalled-by-TC cycles, L1 (TCP) accesses and L2 requests, UTCL1 translation
# hits / misses (the page and record pools are 10-20 GB of random lines).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-extras --steps 10 --warmup 2"}
timeout -k 10 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-include-regex "k_candidates|k_update" -d gpurun_out/pmc_ta -o ta --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_ta.log 2>&1
