# diagnostics: fused-kernel phase split, PMC passes, counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/diag_fused_phases.py > gpurun_out/diag_phases.log 2>&1 || { echo DIAG_FAILED; tail -20 gpurun_out/diag_phases.log; exit 1; }
cat gpurun_out/diag_phases.log | grep -v Warn | tail -8
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
bash tools/gpu_pmc.sh > gpurun_out/pmc_all.log 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc_all.log; exit 1; }
cat gpurun_out/pmc_all.log
