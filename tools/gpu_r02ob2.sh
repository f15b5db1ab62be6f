# OneBlob index shifts: bit-exact tests, configs[1] kernel stats, README throughput benchmarks refreshed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ob2
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_layered.py tests/test_gpu_sample.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/t.txt 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" $OUT/t.txt | head -30; tail -3 $OUT/t.txt; exit 1; }
tail -1 $OUT/t.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/prof_oneblob.py 2 18 64 > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_top.py $OUT/prof > $OUT/top.txt; head -4 $OUT/top.txt
timeout -k 10 400 python -u tools/throughput_bench.py --out $OUT/throughput.json > $OUT/tp.txt 2>&1 || { echo TP_FAILED; tail -20 $OUT/tp.txt; exit 1; }
tail -14 $OUT/tp.txt | cut -c1-200
echo OB2_OK
