#!/bin/bash
# round 6 final build: PMC passes of the headline bench (HBM bytes per launch of
# k_candidates / k_update / k_gather_particles), summarised by scripts/pmc_summary.py
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PMC_OUT=gpurun_out/pmc_v6 bash scripts/pmc_round.sh || { echo pmc failed; exit 5; }
ls gpurun_out/pmc_v6
