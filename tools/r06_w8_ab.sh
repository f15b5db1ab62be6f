# r06: 8-wave fused-kernel workgroups (one per CU: half the network-gradient slabs) vs 4 (two per CU),
# an A/B of two builds of the same tree (TCNN_LIB_PATH selects the 8-wave build), alternating
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_w8}; mkdir -p $D
for v in 4 8 4 8; do
  if [ $v = 8 ]; then export TCNN_LIB_PATH=$PWD/neuralbtf-tiny-cuda-nn_amd/lib_ab/libtcnn_mi355x.so; else unset TCNN_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/bench_$v.log 2>&1 || { tail -5 $D/bench_$v.log; exit 1; }
  timeout -k 10 200 python3 tools/dp_floor.py --schedules plain --steps 400 --batch-log2 15 --out $D/floor_$v.json > $D/floor_$v.log 2>&1 || { tail -5 $D/floor_$v.log; exit 1; }
  python3 -c "
import json
b=[json.loads(l) for l in open('$D/bench_$v.log') if l.startswith('{')][0]
f=json.load(open('$D/floor_$v.json'))['rows'][0]['gpu_us_per_step']
print('waves $v', round(b['value']), {k: round(x*1000,2) for k,x in b['phase_ms'].items() if isinstance(x,float)}, '2^15 %.2f' % f)"
done
