# branch-free in-range grid index in the fused kernel: parity + A/B (TCNN_NO_INRANGE_INDEX=1 = off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fixtures.py tests/test_gpu_grid_large.py tests/test_gpu_edge_cases.py tests/test_gpu_dp.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_r.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_r.log | head -40; exit 1; }
tail -1 gpurun_out/t_r.log
for k in 1 2; do
  VARIANTS="cur" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
  echo "== inrange off"
  TCNN_NO_INRANGE_INDEX=1 VARIANTS="cur" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
done
