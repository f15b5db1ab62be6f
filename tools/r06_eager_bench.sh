# r06: default bench (2^18) with the fused kernel's eager schedule forced on / off, alternating
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/r06_eager_bench; mkdir -p $D
for v in on off on off on off; do
  TCNN_FUSED_EAGER=$([ $v = on ] && echo 1 || echo 0) timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/bench_$v.log 2>&1 || { tail -5 $D/bench_$v.log; exit 1; }
  python3 -c "
import json
b=[json.loads(l) for l in open('$D/bench_$v.log') if l.startswith('{')][0]
print('$v', round(b['value']), {k: round(x*1000,2) for k,x in b['phase_ms'].items() if isinstance(x,float)})"
done
