# r06: grid-backward work plan A/B (TCNN_GRID_BWD_PLAN=range|feature, default = by batch) on one box:
# the 2^15 per-rank floor, the default bench (2^18) and configs[3] (2^20), each plan forced, then default
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_plan}; mkdir -p $D
for plan in range feature default; do
  if [ $plan = default ]; then unset TCNN_GRID_BWD_PLAN; else export TCNN_GRID_BWD_PLAN=$plan; fi
  timeout -k 10 200 python3 tools/dp_floor.py --schedules plain --steps 400 --batch-log2 15 --out $D/floor_$plan.json > $D/floor_$plan.log 2>&1 || { tail -5 $D/floor_$plan.log; exit 1; }
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/bench_$plan.log 2>&1 || { tail -5 $D/bench_$plan.log; exit 1; }
  timeout -k 10 200 python3 tools/c3_time.py > $D/c3_$plan.json 2> $D/c3_$plan.err || { tail -5 $D/c3_$plan.err; exit 1; }
  python3 -c "
import json
f=json.load(open('$D/floor_$plan.json'))['rows'][0]['gpu_us_per_step']
b=[json.loads(l) for l in open('$D/bench_$plan.log') if l.startswith('{')][0]
c=json.load(open('$D/c3_$plan.json'))
print('$plan', '2^15 %.2f us' % f, '2^18 %.0f steps/s' % b['value'], {k: round(v*1000,2) for k,v in b['phase_ms'].items() if isinstance(v,float)}, 'configs3 %.0f steps/s' % c['steps_per_s'])"
done
