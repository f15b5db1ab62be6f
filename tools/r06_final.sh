# r06 end of round on the final tree: GPU suite, smoke, default bench, rocprof kernel stats of the bench,
# PMC traffic + MFMA passes, the per-rank curve (plain + loopback peer step), configs[3], torch A/B
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_final}; mkdir -p $D
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $D/tests.log 2>&1 || { grep -E "FAILED|Error" $D/tests.log | head -20; tail -3 $D/tests.log; exit 1; }
  tail -1 $D/tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -10 $D/smoke.log; exit 1; }
  tail -2 $D/smoke.log
fi
timeout -k 10 300 python3 bench.py > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | cut -c1-240
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --no-cpu-baseline --no-profile --steps 200 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cp "$f" $D/kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$D/kernel_stats.csv')))[:5]: print('%-60s %6s %9.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1000))"
PMC_OUT=$D/pmc bash tools/gpu_pmc.sh tools/pmc_groups.txt > $D/pmc.txt 2>&1 || { tail -5 $D/pmc.txt; exit 1; }
python3 tools/pmc_traffic.py $D/pmc $D/pmc_traffic.json "$(python3 bench.py --print-workload)" > $D/pmc_traffic.log 2>&1 || { tail -5 $D/pmc_traffic.log; exit 1; }
PMC_OUT=$D/pmc_mfma bash tools/gpu_pmc.sh tools/pmc_groups_mfma.txt > $D/pmc_mfma.txt 2>&1 || { tail -5 $D/pmc_mfma.txt; exit 1; }
OUT=$(basename $D)/curve bash tools/r06_curve.sh || exit 1
timeout -k 10 200 python3 tools/c3_time.py > $D/c3.json 2> $D/c3.err || { tail -5 $D/c3.err; exit 1; }
cat $D/c3.json | cut -c1-200
timeout -k 10 300 python3 tools/torch_step_ab.py --out $D/torch_ab.json > $D/torch_ab.log 2>&1 || { tail -5 $D/torch_ab.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/torch_ab.json')); print({k:[round(r['step_us'],1) for r in v] for k,v in d['runs'].items()}, round(d['trainer_step_us'],1))"
