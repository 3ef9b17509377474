#!/bin/bash
# SQ stall breakdown (one counter group, no traces) for the update kernels:
# WAVE_CYCLES = WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY
# (issue stalls) + ACTIVE_INST_ANY, in quad-cycles (MI355X_MICROARCH.md).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline"}
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "k_candidates|k_update|k_gather|k_sweep" -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq.log 2>&1
