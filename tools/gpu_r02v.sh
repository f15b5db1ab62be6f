# in-range index with the stride-loop break mirrored (log2T=19 levels qualify): parity + T19 / headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid_large.py tests/test_gpu_parity.py tests/test_gpu_fixtures.py tests/test_gpu_layered.py tests/test_gpu_graph.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_v.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_v.log | head -40; exit 1; }
tail -1 gpurun_out/t_v.log
for e in "" 1; do
  TCNN_NO_INRANGE_INDEX=$e timeout -k 10 200 python3 bench.py --no-cpu-baseline --log2-hashmap-size 19 --per-level-scale 2.0 > gpurun_out/b19.json 2>gpurun_out/b19.err || { echo B19_FAILED; tail -5 gpurun_out/b19.err; exit 1; }
  TCNN_NO_INRANGE_INDEX=$e timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/b15.json 2>gpurun_out/b15.err || { echo B15_FAILED; exit 1; }
  python3 -c "import json; a=json.load(open('gpurun_out/b19.json')); b=json.load(open('gpurun_out/b15.json')); print('noinrange=[$e] T19', a['value'], a['phase_ms']['fused_grid_mlp_fwd_loss_bwd'], 'T15', b['value'])"
done
