# round-2: template API consumer, sample on albert, full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_template_api.py tests/test_gpu_sample.py tests/test_gpu_cpp_api.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_tpl.log 2>&1 || { echo TPL_FAILED; tail -60 gpurun_out/t_tpl.log; exit 1; }
tail -3 gpurun_out/t_tpl.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
