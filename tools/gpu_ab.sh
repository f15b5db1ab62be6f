# A/B of tuning knobs on the bench; tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ab_$n.log 2>&1 || { echo BENCH_FAILED $n; tail -20 gpurun_out/ab_$n.log; exit 1; }
  grep '^{' gpurun_out/ab_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value']), {k: round(v*1000,1) for k,v in d['phase_ms'].items() if k!='sampled_steps'})"
}
run c9 TCNN_GRID_BWD_CHUNKS=9
run c8 TCNN_GRID_BWD_CHUNKS=8
run c7 TCNN_GRID_BWD_CHUNKS=7
run c9scalar TCNN_GRID_BWD_CHUNKS=9 TCNN_ADAM_SCALAR=1
run c8scalar TCNN_GRID_BWD_CHUNKS=8 TCNN_ADAM_SCALAR=1
