# r05: full GPU suite, W128 tile A/B (32 vs 64 samples), configs[3] kernel stats + tile PMC passes
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_tile2}; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests} > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
TCNN_TILE_SAMPLES=32 timeout -k 10 200 python3 tools/tile_ts_ab.py > $D/ab32.log 2>&1 || { tail -5 $D/ab32.log; exit 1; }
timeout -k 10 200 python3 tools/tile_ts_ab.py > $D/ab64.log 2>&1 || { tail -5 $D/ab64.log; exit 1; }
cat $D/ab32.log $D/ab64.log | grep '^{' | cut -c1-150
OUT=${OUT:-r05_tile2}/tp bash tools/r05_tile_prof.sh
