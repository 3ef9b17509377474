#!/bin/bash
# A/B of environment settings on the config-3 bench (one library):
#   bash scripts/ab_env.sh "" "FS2_FLUSH_MB=256" ...   ("" = no extra setting)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i + 1))
  env $e timeout -k 10 300 python3 bench.py --steps 30 --warmup 2 --no-cpu-baseline --no-extras ${AB_ARGS:-} > gpurun_out/abe_$i.log 2>&1 || { echo "[$e] failed"; tail -5 gpurun_out/abe_$i.log; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abe_$i.log').read().strip().splitlines()[-1]); k=d['extra']['kernels']; print('[$e]', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', {n: round(v['ms_per_launch'],4) for n, v in k.items()}, 'reduce+resample', round(d['extra']['reduce_and_resample_ms'],4))"
done
