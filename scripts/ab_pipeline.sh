#!/bin/bash
# A/B of the pipelined headline (two scans in flight) against step() one at a time,
# and of variants of the speculative pass (libfs2_<tag>.so built with build.py --variant), same box:
# repeated short bench runs, one JSON summary line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/ab_pipeline.txt
: > $OUT
VARIANTS=${VARIANTS:-"default:pipe default:sync mask8:pipe mask4:pipe"}
for rep in 1 2 3; do
  for v in $VARIANTS; do
    set -- ${v//:/ }
    lib=fast-slam_amd/lib/libfs2.so; [ "$1" != default ] && lib=fast-slam_amd/lib/libfs2_$1.so
    extra=""; [ "$2" = pipe ] && extra="--pipelined"
    FS2_LIB=$lib GPU_MAX_HW_QUEUES=${3:-4} timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras $extra > gpurun_out/ab_run.log 2>&1 || { echo "run $v failed"; tail -5 gpurun_out/ab_run.log; exit 3; }
    tail -1 gpurun_out/ab_run.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$rep', '$1', '$2', 'q${3:-4}', round(d['ms_per_step'],4), round(d['value']/1e9,3), 'tail', round(e['reduce_and_resample_ms'],4), 'kupd', round(d['roofline']['ms_per_launch'],4), 'kcand', round(e['kernels']['k_candidates']['ms_per_launch'],4), 'res', e['resamples'], 'opened', round(e['pages_opened_per_particle_scan'],3))" >> $OUT
    tail -1 $OUT
  done
done
