# r05: configs[3] kernel stats + tile-kernel PMC passes (TS env: TCNN_TILE_SAMPLES setting)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_tprof}; mkdir -p $D
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c3 -- python3 tools/prof_configs3.py > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 1; }
f=$(find $D/prof -name '*kernel_stats.csv' | head -1); cp "$f" $D/kernel_stats.csv; cut -d, -f1-4 "$f" | head -6
STEPS=3 PMC_OUT=$D/pmc PMC_CMD="tools/prof_configs3.py" PMC_FILTER=k_mlp_tile bash tools/gpu_pmc.sh tools/pmc_tile_groups.txt > $D/pmc.txt 2>&1 || { tail -5 $D/pmc.txt; exit 1; }
cat $D/pmc.txt
