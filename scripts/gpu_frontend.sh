set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fe_tests.log 2>&1
rc=$?; echo "frontend pytest rc=$rc"; tail -15 gpurun_out/fe_tests.log
[[ $rc -ne 0 ]] && exit $rc
timeout -k 10 300 python -u scripts/bench_frontend.py > gpurun_out/fe_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/fe_bench.log; exit 4; }
tail -1 gpurun_out/fe_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/feprof -o run -- python3 scripts/bench_frontend.py --reps 3 --cpu-scans 2 > gpurun_out/fe_prof.log 2>&1 || { echo prof failed; tail -20 gpurun_out/fe_prof.log; exit 5; }
python scripts/prof_summary.py gpurun_out/feprof gpurun_out/fe_prof_summary.txt "front-end" > /dev/null && head -20 gpurun_out/fe_prof_summary.txt
