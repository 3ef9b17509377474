#!/bin/bash
# round 6 (re-run on the final build): the 8-process rehearsal (8 ranks on one GPU, shm transport, 300 K particles
# per rank), now with the bytes each rank receives and the exposed exchange time
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --gpus 8 --share-gpu --particles 300000 --steps 8 --warmup 2 \
    --no-cpu-baseline > gpurun_out/bench_g8.log 2>&1
rc=$?
grep '^{' gpurun_out/bench_g8.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); print(json.dumps(d['extra'].get('migration'), indent=1))"
exit $rc
