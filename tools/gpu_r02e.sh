# round-2: frozen-fixture GPU parity + the full GPU suite (after the strided-RNG fix)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixtures.py tests/test_gpu_template_api.py -v --timeout 120 --timeout-method thread > gpurun_out/t_fix.log 2>&1 || { echo FIX_FAILED; grep -E "PASS|FAIL|Error|assert" gpurun_out/t_fix.log | head -60; exit 1; }
tail -3 gpurun_out/t_fix.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
