# hipGraph step replay: parity + bench with / without graph + small-batch throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_u.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_u.log | head -40; exit 1; }
tail -1 gpurun_out/t_u.log
for k in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --graph > gpurun_out/b_graph.json 2>gpurun_out/b_graph.err || { echo BG_FAILED; tail -5 gpurun_out/b_graph.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/b_eager.json 2>gpurun_out/b_eager.err || { echo BE_FAILED; exit 1; }
python3 -c "import json; g=json.load(open('gpurun_out/b_graph.json')); e=json.load(open('gpurun_out/b_eager.json')); print('graph', g['value'], 'eager', e['value'])"
done
for B in 14 16; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --graph --batch-log2 $B > gpurun_out/b_graph.json 2>gpurun_out/b_graph.err || { echo BG_FAILED; tail -5 gpurun_out/b_graph.err; exit 1; }
timeout -k 10 200 python3 bench.py --no-cpu-baseline --batch-log2 $B > gpurun_out/b_eager.json 2>gpurun_out/b_eager.err || { echo BE_FAILED; exit 1; }
python3 -c "import json; g=json.load(open('gpurun_out/b_graph.json')); e=json.load(open('gpurun_out/b_eager.json')); print('B=2^$B graph', g['value'], 'eager', e['value'])"
done
