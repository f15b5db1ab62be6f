# Headline (config_hash, B=2^18) profile: kernel stats + PMC traffic / instruction mix
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof_h
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_h -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_h.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_h.log; exit 1; }
tail -1 gpurun_out/prof_h.log
python3 tools/prof_top.py gpurun_out/prof_h > gpurun_out/prof_h_top.txt; head -8 gpurun_out/prof_h_top.txt
PMC_OUT=gpurun_out/pmc_h bash tools/gpu_pmc.sh tools/pmc_groups.txt > gpurun_out/pmc_h.txt 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_h.txt; exit 1; }
echo PMC_OK
