# in-range index in the AoS grid forward: parity + configs[3] kernel stats with / without
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixtures.py tests/test_gpu_grid_large.py tests/test_gpu_layered.py tests/test_gpu_grid_options.py tests/test_gpu_parity.py tests/test_gpu_api_surface.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_s.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_s.log | head -40; exit 1; }
tail -1 gpurun_out/t_s.log
for v in on off; do
  rm -rf gpurun_out/prof_c3_$v
  if [ $v = off ]; then export TCNN_NO_INRANGE_INDEX=1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$v -o run -- python3 tools/prof_configs3.py > gpurun_out/prof_c3_$v.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_c3_$v.log; exit 1; }
  echo "== $v"; python3 tools/prof_top.py gpurun_out/prof_c3_$v > gpurun_out/prof_c3_$v.txt; head -5 gpurun_out/prof_c3_$v.txt
done
