# Round-2 record on the final tree: full GPU suite, smoke, bench (+ CPU baseline), rocprof stats of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/rec2
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { echo TESTS_FAILED; grep -E "^FAILED|Error" $OUT/gpu_tests.txt | head -20; tail -3 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof_bench.log; exit 1; }
python3 tools/prof_top.py $OUT/prof > $OUT/prof_top.txt; head -5 $OUT/prof_top.txt
echo REC_OK
