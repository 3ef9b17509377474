#!/bin/bash
# A/B of library builds on the config-3 bench: bash scripts/ab_bench.sh a b c
# (fast-slam_amd/lib/libfs2_<tag>.so each; one bench run per build, no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in "$@"; do
  lib=fast-slam_amd/lib/libfs2_$t.so; [ "$t" = main ] && lib=fast-slam_amd/lib/libfs2.so; FS2_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$t.log 2>&1 || { echo "$t failed"; tail -5 gpurun_out/ab_$t.log; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$t.log').read().strip().splitlines()[-1]); k=d['extra']['kernels']; print('$t', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', {n: round(v['ms_per_launch'],4) for n, v in k.items()}, 'reduce+resample', round(d['extra']['reduce_and_resample_ms'],4))"
done
