# r05: tile-engine GPU tests + the tile A/B table (tools/tile_ts_ab.py) on the current tree
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_tq}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_layered.py tests/test_gpu_tile_engine.py tests/test_gpu_graph.py tests/test_gpu_dp_peer.py > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 200 python3 tools/tile_ts_ab.py > $D/ab.log 2>&1 || exit 1
grep '^{' $D/ab.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['case'][:40], round(d['steps_per_s']))"
