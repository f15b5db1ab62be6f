cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/r05_b; mkdir -p $D
run() { c=$1; TCNN_GRID_BWD_CHUNKS=$c timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c$c -o run -- python3 tools/dp_floor.py --schedules plain > $D/c$c.log 2>&1 && python3 tools/prof_top.py $D/c$c | head -5 && grep schedule $D/c$c.log | cut -c1-120; }
run 1 && run 2 && run 4 && run 8 && TCNN_DEBUG_GRID_TIMES=1 LOG2B=15 STEPS=3 timeout -k 10 120 python3 tools/diag_grid_times.py 2> $D/gt15.txt > $D/gt15.out && echo GT_OK
