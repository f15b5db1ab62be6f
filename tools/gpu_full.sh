# Round measurement: GPU parity tests, the default bench (with CPU baseline), rocprofv3 kernel-trace
# stats of the same command, PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hits / SQ) -> gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/prof.log; exit 1; }
python3 tools/prof_top.py gpurun_out/prof
bash tools/gpu_pmc.sh > gpurun_out/pmc_passes.log 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_passes.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc_run gpurun_out/pmc_traffic.json
