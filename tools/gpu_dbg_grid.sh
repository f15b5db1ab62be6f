cd $GRAFT_REPO_ROOT
TCNN_DEBUG_GRID_TIMES=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/dbg_grid.log 2>&1 || { tail -20 gpurun_out/dbg_grid.log; exit 1; }
grep -A 44 "grid_bwd:" gpurun_out/dbg_grid.log | tail -44 | awk 'NR<=2 || /item (0|5|6|25):/ || /tail wg (0|1|15):/'
