#!/bin/bash
# rocprofv3 kernel stats of the config-3 bench for several library builds:
# bash scripts/ab_prof.sh a b ...  (fast-slam_amd/lib/libfs2_<tag>.so; "main" = libfs2.so)
# -> gpurun_out/abprof_<tag>.txt per build (scripts/prof_summary.py format)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in "$@"; do
  lib=fast-slam_amd/lib/libfs2_$t.so; [ "$t" = main ] && lib=fast-slam_amd/lib/libfs2.so
  rm -rf /tmp/abprof_$t
  FS2_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/abprof_$t -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/abprof_$t.log 2>&1 || { echo "$t failed"; tail -5 gpurun_out/abprof_$t.log; exit 4; }
  python3 scripts/prof_summary.py /tmp/abprof_$t gpurun_out/abprof_$t.txt "$t" > /dev/null || exit 5
  echo "== $t"; grep -E "k_mark|k_sweep|k_update|k_candidates" gpurun_out/abprof_$t.txt
done
