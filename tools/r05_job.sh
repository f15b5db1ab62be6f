# r05 scratch job: GPU tests given as $1 (pytest node ids), then grid-backward phase times at 2^15 / 2^18
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_job}; mkdir -p $D
timeout -k 10 600 python -u -m pytest $1 -m gpu -x -v --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -15 $D/tests.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$GT" ]; then
  for b in 15 18; do TCNN_DEBUG_GRID_TIMES=1 LOG2B=$b STEPS=3 timeout -k 10 120 python3 tools/diag_grid_times.py 2> $D/gt$b.txt > $D/gt$b.out || exit 1; done
  grep -E "item  (0|6|20)|tail wg 0|span" $D/gt15.txt $D/gt18.txt | tail -16
fi
