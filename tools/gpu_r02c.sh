# PMC passes of the log2T=19 step (traffic + latency groups)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export BENCH_EXTRA="--log2-hashmap-size 19 --per-level-scale 2.0"
PMC_OUT=gpurun_out/pmc19 bash tools/gpu_pmc.sh tools/pmc_groups.txt > gpurun_out/pmc19_traffic.txt 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/pmc19_traffic.txt; exit 1; }
PMC_OUT=gpurun_out/pmc19l bash tools/gpu_pmc.sh tools/pmc_groups_latency.txt > gpurun_out/pmc19_latency.txt 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc19_latency.txt; exit 1; }
cat gpurun_out/pmc19_traffic.txt gpurun_out/pmc19_latency.txt
