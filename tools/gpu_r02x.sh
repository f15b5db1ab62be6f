# Re-entry check after container re-creation: full GPU suite, smoke, default bench. Output: gpurun_out/x/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/x
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { echo TESTS_FAILED; grep -E "^FAILED|Error" $OUT/gpu_tests.txt | head -20; tail -3 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
echo X_OK
