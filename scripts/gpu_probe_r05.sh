#!/bin/bash
# Round-5 probes: cross-process sharing (scripts/ipc_probe.sh), the growth after
# closed handles (scripts/g8_refs_probe.py with FS2_TRACE), then the given tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ipc_probe.sh > gpurun_out/ipc_probe.log 2>&1; echo probes rc=$?
FS2_TRACE=1 timeout -k 10 300 python3 scripts/g8_refs_probe.py 3 > gpurun_out/g8_probe.log 2> gpurun_out/g8_trace.log || { echo g8 failed; exit 4; }
grep "fs2 vmm" gpurun_out/g8_trace.log | sort -t' ' -k5 -n | tail -4
grep "profile rank0\|scan [0-9] start" gpurun_out/g8_probe.log | awk '{print $0}' | cut -c1-160 | tail -12
TESTS=${TESTS:-tests/test_gpu_pool_growth.py} bash scripts/gpu_session.sh tests
