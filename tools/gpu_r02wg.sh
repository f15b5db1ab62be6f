# tile kernel workgroups per CU (TCNN_TILE_WG_PER_CU): parity at 2, engine A/B at 1 / 2 / 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/wg
rm -rf $OUT; mkdir -p $OUT
TCNN_TILE_WG_PER_CU=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_layered.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/t.txt 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" $OUT/t.txt | head -20; exit 1; }
tail -1 $OUT/t.txt
for k in 1 2 3; do
TCNN_TILE_WG_PER_CU=$k timeout -k 10 200 python -u tools/engine_ab.py --iters 20 > $OUT/ab$k.txt 2>&1 || { echo AB_FAILED; tail -5 $OUT/ab$k.txt; exit 1; }
echo "k=$k"; grep '^{' $OUT/ab$k.txt | python3 -c "
import sys, json
for d in map(json.loads, sys.stdin): print('  ', d['case'][:40], round(d['tile']['steps_per_s']))"
done
echo WG_OK
