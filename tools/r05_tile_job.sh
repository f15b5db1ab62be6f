# r05: tile engine tests + 32 vs 64 samples per tile A/B + configs[3] kernel stats
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_tile}; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_tile_engine.py} > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
TCNN_TILE_SAMPLES=32 timeout -k 10 200 python3 tools/tile_ts_ab.py > $D/ab32.log 2>&1 || { tail -5 $D/ab32.log; exit 1; }
timeout -k 10 200 python3 tools/tile_ts_ab.py > $D/ab64.log 2>&1 || { tail -5 $D/ab64.log; exit 1; }
cat $D/ab32.log $D/ab64.log | cut -c1-160
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c3 -- python3 tools/prof_configs3.py > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -8
