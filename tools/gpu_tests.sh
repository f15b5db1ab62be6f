# GPU parity tests only (verbose log under gpurun_out/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -40 gpurun_out/gpu_tests.log
