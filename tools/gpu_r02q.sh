# XCD-aware chunk mapping + early position prefetch: parity, phase times, A/B, 9-chunk variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TCNN_DEBUG_POISON=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_grid_large.py tests/test_gpu_parity.py tests/test_gpu_fixtures.py tests/test_gpu_dp.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_q.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_q.log | head -40; exit 1; }
tail -1 gpurun_out/t_q.log
TCNN_DEBUG_GRID_TIMES=1 timeout -k 10 120 python3 tools/diag_grid_times.py 2> gpurun_out/grid_times.txt || { echo DIAG_FAILED; exit 1; }
tail -30 gpurun_out/grid_times.txt | head -4
VARIANTS="cur v1" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
echo "== 9 chunks"
TCNN_GRID_BWD_CHUNKS=9 VARIANTS="cur" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
