#!/bin/bash
# PMC passes (one counter group per pass; no --sys/--hip trace): HBM bytes of
# k_candidates / k_update / k_copy_maps from FETCH_SIZE / WRITE_SIZE, plus a FETCH_SIZE calibration on the
# layout microbenchmark whose byte count is known (MI355X_MICROARCH.md §HBM).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-extras"}
OUT=${PMC_OUT:-gpurun_out}          # one directory per workload (summarised from it)
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_soa|k_desc8|k_lines128" -d $OUT/pmc_cal -o cal --output-format csv -- ./scripts/ubench_layout > $OUT/pmc_cal.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_candidates|k_update|k_gather_particles" -d $OUT/pmc_fetch -o fetch --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_candidates|k_update|k_gather_particles" -d $OUT/pmc_write -o write --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1
# summarise after the outputs are merged back: python3 scripts/pmc_summary.py $OUT <workload> <tag>
