# register-resident grid backward: parity (poisoned allocations), phase times, A/B vs _v1wt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TCNN_DEBUG_POISON=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_grid_large.py tests/test_gpu_parity.py tests/test_gpu_fixtures.py tests/test_gpu_layered.py tests/test_gpu_grid_options.py tests/test_gpu_grid_input.py tests/test_gpu_dp.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_p.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_p.log | head -40; exit 1; }
tail -1 gpurun_out/t_p.log
TCNN_DEBUG_GRID_TIMES=1 timeout -k 10 120 python3 tools/diag_grid_times.py 2> gpurun_out/grid_times.txt || { echo DIAG_FAILED; exit 1; }
tail -30 gpurun_out/grid_times.txt | head -6
VARIANTS="cur v1 cur v1" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
