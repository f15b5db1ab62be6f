# r05: per-rank step floor at the shard sizes of N = 1, 2, 4, 8 (2^18 / N points; plain and peer on one rank),
# the default bench, and rocprof kernel stats of the bench at 2^18
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_curve}; mkdir -p $D
for lb in 18 17 16 15; do
  timeout -k 10 120 python3 tools/dp_floor.py --schedules plain,peer --steps 400 --batch-log2 $lb --out $D/floor_$lb.json > $D/floor_$lb.log 2>&1 || { tail -5 $D/floor_$lb.log; exit 1; }
  python3 -c "import json; d=json.load(open('$D/floor_$lb.json')); [print($lb, r['schedule'], round(r['gpu_us_per_step'],2), round(r['host_issue_us_per_step'],2)) for r in d['rows']]"
done
timeout -k 10 200 python3 bench.py > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --no-cpu-baseline --no-profile --steps 200 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cp "$f" $D/kernel_stats.csv; cut -d, -f1-4 "$f" | head -5 | cut -c1-60,150-
