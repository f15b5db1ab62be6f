# A/B of tuning/diagnostic knobs on the bench (no tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ab_$n.log 2>&1 || { echo BENCH_FAILED $n; tail -20 gpurun_out/ab_$n.log; exit 1; }
  grep '^{' gpurun_out/ab_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['value']), {k: round(v*1000,1) for k,v in d['phase_ms'].items() if k!='sampled_steps'})"
}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  run $name $envs
done
