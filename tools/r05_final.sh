# r05 end of round on the final tree: GPU suite, smoke, default bench, rocprof kernel stats of the bench,
# PMC traffic + MFMA passes, the per-rank floor at 2^15 (plain + peer)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_final}; mkdir -p $D
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -10 $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
timeout -k 10 300 python3 bench.py > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | cut -c1-240
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --no-cpu-baseline --no-profile --steps 200 > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cp "$f" $D/kernel_stats.csv
PMC_OUT=$D/pmc bash tools/gpu_pmc.sh tools/pmc_groups.txt > $D/pmc.txt 2>&1 || { tail -5 $D/pmc.txt; exit 1; }
PMC_OUT=$D/pmc_mfma bash tools/gpu_pmc.sh tools/pmc_groups_mfma.txt > $D/pmc_mfma.txt 2>&1 || { tail -5 $D/pmc_mfma.txt; exit 1; }
timeout -k 10 120 python3 tools/dp_floor.py --schedules plain,peer --steps 400 --batch-log2 15 --out $D/floor15.json > $D/floor15.log 2>&1 || { tail -5 $D/floor15.log; exit 1; }
python3 -c "import json; d=json.load(open('$D/floor15.json')); [print(r['schedule'], round(r['gpu_us_per_step'],2)) for r in d['rows']]"
