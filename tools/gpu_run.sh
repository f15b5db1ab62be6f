set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*"; python3 tools/prof_top.py gpurun_out/prof
