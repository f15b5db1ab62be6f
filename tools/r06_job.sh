# r06 scratch job: GPU tests given as $1 (pytest node ids, "-" for none), then the per-rank floor for the
# schedules in $SCHED (default plain,peer) at 2^$LOG2B points (default 15), then optionally ($BENCH) the
# default bench
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_job}; mkdir -p $D
if [ "$1" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $1 -m gpu -x -v --timeout 240 --timeout-method thread > $D/tests.log 2>&1; rc=$?
  tail -4 $D/tests.log
  [ $rc -eq 0 ] || { grep -E "Error|error|assert" $D/tests.log | head -20; exit $rc; }
fi
for lb in ${LOG2B:-15}; do
  timeout -k 10 240 python3 tools/dp_floor.py --schedules ${SCHED:-plain,peer} --steps 400 --batch-log2 $lb --out $D/floor_$lb.json > $D/floor_$lb.log 2>&1 || { tail -5 $D/floor_$lb.log; exit 1; }
  python3 -c "import json; d=json.load(open('$D/floor_$lb.json')); [print($lb, r['schedule'][:40], round(r['gpu_us_per_step'],2), round(r['host_issue_us_per_step'],2)) for r in d['rows']]"
done
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
  grep '^{' $D/bench.log | cut -c1-200
fi
if [ -n "$PROF" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/dp_floor.py --schedules $PROF --steps 400 --batch-log2 ${LOG2B:-15} > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
  f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cp "$f" $D/kstats.csv
  python3 -c "
import csv
for r in list(csv.DictReader(open('$D/kstats.csv')))[:9]: print('%-60s %6s %9.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1000))"
fi
