# A/B timing of the streamed tile shapes only (after a kernel change), plus the layered parity file
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/z2
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_layered.py tests/test_gpu_fixtures.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/t.txt 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" $OUT/t.txt | head -30; tail -3 $OUT/t.txt; exit 1; }
tail -1 $OUT/t.txt
timeout -k 10 300 python -u tools/engine_ab.py > $OUT/ab.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab.txt; exit 1; }
grep "^{" $OUT/ab.txt | cut -c1-260
echo Z_OK
