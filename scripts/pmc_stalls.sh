#!/bin/bash
# Where the update kernels' wave time goes (round 5, for the next round's work): three
# rocprofv3 --pmc passes of at most 8 SQ counters each over the default bench
# (no trace domains), per dispatch of k_candidates / k_update / k_gather_particles.
# Summarise with: python3 scripts/pmc_stalls.py gpurun_out/pmc_stalls
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_stalls}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-extras"}
KERN="k_candidates|k_update|k_gather_particles"
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 400 rocprofv3 --pmc "$@" --kernel-include-regex "$KERN" -d $OUT/$name -o $name \
    --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
pass b SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_TRANS_F64 SQ_LEVEL_WAVES
pass c SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
echo "pmc stalls done"
