# r06: configs[3] with the in-kernel grid encode (default) vs the separate AoS pass (TCNN_TILE_GENC=0),
# then rocprof kernel stats of the default
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_c3}; mkdir -p $D
for v in 1 0 1 0; do
  TCNN_TILE_GENC=$v timeout -k 10 200 python3 tools/c3_time.py >> $D/ab.jsonl 2> $D/ab_err.log || { tail -5 $D/ab_err.log; exit 1; }
  tail -1 $D/ab.jsonl | cut -c1-200
done
STEPS=30 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/prof_configs3.py > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cp "$f" $D/kstats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$D/kstats.csv')))[:8]: print('%-70s %6s %9.2f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1000))"
