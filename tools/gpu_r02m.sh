# Rounding-barrier change: fused/grid-forward parity + headline timing vs round 1 on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fixtures.py tests/test_gpu_parity.py tests/test_gpu_grid_large.py tests/test_gpu_layered.py tests/test_gpu_edge_cases.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_m.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_m.log | head -40; exit 1; }
tail -2 gpurun_out/t_m.log
VARIANTS="cur r01" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
