# r06: the fused kernel's small-batch schedule (EAGER: all corner loads of a slice before the first
# combine) vs the per-level schedule, one build, TCNN_FUSED_EAGER=0/1 (default: eager while every wave has
# at most one slice): bit identity (tools/ab_bitident.py), GPU tests, then the plain step at 2^15..2^18
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/r06_eager; mkdir -p $D
timeout -k 10 200 python3 -u tools/ab_bitident.py > $D/bit_auto.log 2>&1 || { tail -5 $D/bit_auto.log; exit 1; }
TCNN_FUSED_EAGER=0 timeout -k 10 200 python3 -u tools/ab_bitident.py > $D/bit_off.log 2>&1 || { tail -5 $D/bit_off.log; exit 1; }
TCNN_FUSED_EAGER=1 timeout -k 10 200 python3 -u tools/ab_bitident.py > $D/bit_on.log 2>&1 || { tail -5 $D/bit_on.log; exit 1; }
for v in auto off on; do echo $v $(grep case $D/bit_$v.log | awk '{print $4}'); done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
  tail -1 $D/tests.log
fi
for rep in 1 2; do
  for v in off on; do
    for lb in 15 16 17 18; do
      TCNN_FUSED_EAGER=$([ $v = on ] && echo 1 || echo 0) timeout -k 10 120 python3 tools/dp_floor.py --schedules plain --steps 400 --batch-log2 $lb --out $D/${v}_${lb}_$rep.json > $D/${v}_${lb}_$rep.log 2>&1 || { tail -5 $D/${v}_${lb}_$rep.log; exit 1; }
    done
    python3 -c "
import json
print('$v', $rep, [(lb, round(json.load(open('$D/${v}_%d_$rep.json' % lb))['rows'][0]['gpu_us_per_step'], 2)) for lb in (15, 16, 17, 18)])"
  done
done
