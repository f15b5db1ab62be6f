# full GPU suite with NaN-poisoned engine allocations, then 8-wave vs 4-wave (HEAD, _v1wt) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TCNN_DEBUG_POISON=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t_poison.log 2>&1; rc=$?
tail -3 gpurun_out/t_poison.log; grep -E "^FAILED" gpurun_out/t_poison.log | head -30
[ $rc -gt 1 ] && { echo SUITE_CRASHED $rc; exit 1; }
VARIANTS="cur v1 cur v1" EXTRA=--no-cpu-baseline bash tools/gpu_ab_r01.sh
