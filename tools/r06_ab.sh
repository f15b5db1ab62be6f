# r06: A/B of the tree's build ("new") against lib_ab ("base", another build of the library): bit identity of
# a few training steps (tools/ab_bitident.py), optionally GPU tests ($TESTS), then alternating default bench
# + the 2^15 per-rank floor
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_pf}; mkdir -p $D
AB=$PWD/neuralbtf-tiny-cuda-nn_amd/lib_ab/libtcnn_mi355x.so
timeout -k 10 200 python3 -u tools/ab_bitident.py > $D/bit_new.log 2>&1 || { tail -5 $D/bit_new.log; exit 1; }
TCNN_LIB_PATH=$AB timeout -k 10 200 python3 -u tools/ab_bitident.py > $D/bit_base.log 2>&1 || { tail -5 $D/bit_base.log; exit 1; }
cat $D/bit_new.log $D/bit_base.log | grep case
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
  tail -2 $D/tests.log
fi
for v in new base new base; do
  if [ $v = base ]; then export TCNN_LIB_PATH=$AB; else unset TCNN_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/bench_$v.log 2>&1 || { tail -5 $D/bench_$v.log; exit 1; }
  timeout -k 10 200 python3 tools/dp_floor.py --schedules plain --steps 400 --batch-log2 15 --out $D/floor_$v.json > $D/floor_$v.log 2>&1 || { tail -5 $D/floor_$v.log; exit 1; }
  python3 -c "
import json
b=[json.loads(l) for l in open('$D/bench_$v.log') if l.startswith('{')][0]
f=json.load(open('$D/floor_$v.json'))['rows'][0]['gpu_us_per_step']
print('$v', round(b['value']), {k: round(x*1000,2) for k,x in b['phase_ms'].items() if isinstance(x,float)}, '2^15 %.2f' % f)"
done
