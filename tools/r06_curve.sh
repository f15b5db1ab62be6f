# r06: per-rank step at the N = 1/2/4/8 shard sizes of the 2^18 batch (plain, and the peer exchange's
# per-rank kernels in loopback at that N: Adam on 1/N of the parameters summing N mirrors, the gather of
# N - 1 shards, every poll), then the rocprof breakdown of the N = 8 loopback step
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_curve}; mkdir -p $D
for lb in 18 17 16 15; do
  n=$((1 << (18 - lb))); s=plain; [ $n -gt 1 ] && s=plain,peerloop$n
  timeout -k 10 200 python3 tools/dp_floor.py --schedules $s --steps 400 --batch-log2 $lb --out $D/floor_$lb.json > $D/floor_$lb.log 2>&1 || { tail -5 $D/floor_$lb.log; exit 1; }
  python3 -c "import json; d=json.load(open('$D/floor_$lb.json')); [print($lb, r['schedule'][:24], round(r['gpu_us_per_step'],2), round(r['host_issue_us_per_step'],2)) for r in d['rows']]"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof8 -o run -- python3 tools/dp_floor.py --schedules peerloop8 --steps 400 --batch-log2 15 > $D/prof8.log 2>&1 || { tail -5 $D/prof8.log; exit 1; }
f=$(find $D/prof8 -name '*kernel_stats.csv' | head -1); cp "$f" $D/kstats_peerloop8.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$D/kstats_peerloop8.csv')))[:7]: print('%-60s %6s %9.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1000))"
