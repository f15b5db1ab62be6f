# r05 A/B of environment switches on the 2^15 (one rank of N=8) and 2^18 steps:
#   bash tools/r05_ab.sh "VAR=a VAR2=b" "VAR=c" ...   (each argument = one variant's env assignments)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_ab}; mkdir -p $D
n=0
for v in "$@"; do
  n=$((n+1))
  echo "== variant $n: $v" | tee -a $D/summary.txt
  env $v timeout -k 10 120 python3 tools/dp_floor.py --schedules plain --steps 400 > $D/v$n.floor.log 2>&1 || { tail -5 $D/v$n.floor.log; exit 1; }
  grep '"plain"' $D/v$n.floor.log | cut -c1-90 | tee -a $D/summary.txt
  env $v timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 400 --no-profile > $D/v$n.bench.log 2>&1 || { tail -5 $D/v$n.bench.log; exit 1; }
  grep '^{' $D/v$n.bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('2^18 steps/s %.0f  ms %.4f' % (d['value'], d['ms_per_step']))" | tee -a $D/summary.txt
done
if [ -n "$GT" ]; then
  env $GT TCNN_DEBUG_GRID_TIMES=1 LOG2B=15 STEPS=3 timeout -k 10 120 python3 tools/diag_grid_times.py 2> $D/gt15.txt > $D/gt15.out || exit 1
  grep -E "item  (0|6|20)|tail wg (0|1)\b|span" $D/gt15.txt | tail -8
fi
