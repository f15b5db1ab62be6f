# Round-2 record: full GPU suite, smoke, bench (+ CPU baseline), rocprof stats, PMC traffic and
# latency passes, fused-kernel phase split, log2T=19 variant bench + stats. Output: gpurun_out/final/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/final
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { echo TESTS_FAILED; grep -E "^FAILED|Error" $OUT/gpu_tests.txt | head -20; tail -3 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof_bench.log; exit 1; }
python3 tools/prof_top.py $OUT/prof > $OUT/prof_top.txt; head -5 $OUT/prof_top.txt
PMC_OUT=$OUT/pmc bash tools/gpu_pmc.sh tools/pmc_groups.txt > $OUT/pmc.txt 2>&1 || { echo PMC_FAILED; tail -5 $OUT/pmc.txt; exit 1; }
PMC_OUT=$OUT/pmc_lat bash tools/gpu_pmc.sh tools/pmc_groups_latency.txt > $OUT/pmc_lat.txt 2>&1 || { echo PMC_LAT_FAILED; tail -5 $OUT/pmc_lat.txt; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc $OUT/pmc_traffic.json && echo pmc ok
timeout -k 10 120 python3 tools/diag_fused_phases.py > $OUT/fused_phases.txt 2>&1 || { echo PHASES_FAILED; tail -5 $OUT/fused_phases.txt; exit 1; }
timeout -k 10 300 python3 bench.py --log2-hashmap-size 19 --per-level-scale 2.0 --no-cpu-baseline > $OUT/bench_t19.json 2> $OUT/bench_t19.err || { echo T19_FAILED; tail -5 $OUT/bench_t19.err; exit 1; }
cut -c1-200 $OUT/bench_t19.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_t19 -o run -- python3 bench.py --log2-hashmap-size 19 --per-level-scale 2.0 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/prof_t19.log 2>&1 || { echo PROF19_FAILED; exit 1; }
python3 tools/prof_top.py $OUT/prof_t19 > $OUT/prof_t19_top.txt; head -5 $OUT/prof_t19_top.txt
echo FINAL_OK
