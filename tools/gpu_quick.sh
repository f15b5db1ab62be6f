# quick GPU iteration: parity tests, a plain bench (no CPU baseline), kernel-trace stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench_quick.log; exit 1; }
grep '^{' gpurun_out/bench_quick.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], d['ms_per_step'], d['phase_ms'], d.get('roofline'))"
rm -rf gpurun_out/prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/prof.log; exit 1; }
python3 tools/prof_top.py gpurun_out/prof
