# r05: tile-engine tests + every tile configuration with 64-sample tiles (default) vs TCNN_TILE_SAMPLES=32
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_tsall}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layered.py tests/test_gpu_tile_engine.py tests/test_gpu_graph.py > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python3 tools/tile_ts_ab.py > $D/ab64.log 2>&1 || exit 1
TCNN_TILE_SAMPLES=32 timeout -k 10 300 python3 tools/tile_ts_ab.py > $D/ab32.log 2>&1 || exit 1
for f in ab64 ab32; do grep '^{' $D/$f.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$f', d['case'][:44], round(d['steps_per_s']))"; done
