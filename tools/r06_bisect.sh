# r06 scratch: bit identity (tools/ab_bitident.py) and the default bench across several builds of the
# library (lib_v*/, lib_ab/ = base)
cd "${GRAFT_REPO_ROOT:-.}"; D=gpurun_out/r06_bisect; mkdir -p $D
P=$PWD/neuralbtf-tiny-cuda-nn_amd
for v in new new2 v1 v2 v3 base; do
  case $v in new|new2) unset TCNN_LIB_PATH;; base) export TCNN_LIB_PATH=$P/lib_ab/libtcnn_mi355x.so;; *) export TCNN_LIB_PATH=$P/lib_$v/libtcnn_mi355x.so;; esac
  timeout -k 10 200 python3 -u tools/ab_bitident.py > $D/bit_$v.log 2>&1 || { tail -5 $D/bit_$v.log; exit 1; }
  echo $v $(grep case $D/bit_$v.log | awk '{print $4}')
done
for v in new v2 v3 base; do
  case $v in new) unset TCNN_LIB_PATH;; base) export TCNN_LIB_PATH=$P/lib_ab/libtcnn_mi355x.so;; *) export TCNN_LIB_PATH=$P/lib_$v/libtcnn_mi355x.so;; esac
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $D/bench_$v.log 2>&1 || { tail -5 $D/bench_$v.log; exit 1; }
  python3 -c "
import json
b=[json.loads(l) for l in open('$D/bench_$v.log') if l.startswith('{')][0]
print('$v', round(b['value']), {k: round(x*1000,2) for k,x in b['phase_ms'].items() if isinstance(x,float)})"
done
