# next-slice position prefetch in the fused kernel: parity + A/B vs HEAD build (_v1wt)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fixtures.py tests/test_gpu_dp.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_t.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_t.log | head -40; exit 1; }
tail -1 gpurun_out/t_t.log
VARIANTS="cur v1 cur v1" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
