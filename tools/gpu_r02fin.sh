# final tree: full GPU suite + smoke + engine A/B (tile default: 2 workgroups per CU where they fit)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/fin
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { echo TESTS_FAILED; grep -E "^FAILED|Error" $OUT/gpu_tests.txt | head -20; tail -3 $OUT/gpu_tests.txt; exit 1; }
tail -1 $OUT/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 200 python -u tools/engine_ab.py --out $OUT/engine_ab.json > $OUT/ab.txt 2>&1 || { echo AB_FAILED; tail -5 $OUT/ab.txt; exit 1; }
grep '^{' $OUT/ab.txt | python3 -c "
import sys, json
for d in map(json.loads, sys.stdin): print('  ', d['case'][:40], round(d['tile']['steps_per_s']), round(d['layered']['steps_per_s']))"
echo FIN_OK
