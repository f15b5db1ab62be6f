# round-2: API-surface tests, full GPU suite, as-file + log2T=19 bench, rocprof of the T=19 step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_grid_large.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_api.log 2>&1 || { echo API_FAILED; tail -60 gpurun_out/t_api.log; exit 1; }
tail -3 gpurun_out/t_api.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_asfile.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench_asfile.log; exit 1; }
grep '^{' gpurun_out/bench_asfile.log | cut -c1-300
timeout -k 10 200 python -u bench.py --no-cpu-baseline --log2-hashmap-size 19 --per-level-scale 2.0 > gpurun_out/bench_t19.log 2>&1 || { echo BENCH19_FAILED; tail -30 gpurun_out/bench_t19.log; exit 1; }
grep '^{' gpurun_out/bench_t19.log | cut -c1-300
rm -rf gpurun_out/prof19
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof19 -o run -- python3 bench.py --no-cpu-baseline --no-profile --log2-hashmap-size 19 --per-level-scale 2.0 --steps 50 > gpurun_out/prof19.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/prof19.log; exit 1; }
python3 tools/prof_top.py gpurun_out/prof19 > gpurun_out/prof19_top.txt; cat gpurun_out/prof19_top.txt
