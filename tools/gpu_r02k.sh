# AoS grid forward rewrite: bit-exactness (fixtures, grid variants, layered/tile parity) + configs[3] timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fixtures.py tests/test_gpu_grid_large.py tests/test_gpu_layered.py tests/test_gpu_grid_options.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_fwd.log 2>&1 || { echo FWD_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_fwd.log | head -40; exit 1; }
tail -2 gpurun_out/t_fwd.log
rm -rf gpurun_out/prof_c3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 tools/prof_configs3.py > gpurun_out/prof_c3.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_c3.log; exit 1; }
python3 tools/prof_top.py gpurun_out/prof_c3 > gpurun_out/prof_c3_top.txt; head -6 gpurun_out/prof_c3_top.txt
