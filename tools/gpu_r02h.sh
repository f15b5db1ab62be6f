# tile engine: parity (layered/api/fixtures tests), then A/B timing vs the layer-wise engine
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_layered.py tests/test_gpu_fixtures.py tests/test_gpu_api_surface.py -v --timeout 200 --timeout-method thread > gpurun_out/t_tile.log 2>&1 || { echo TILE_FAILED; grep -E "PASS|FAIL|Error|assert|error" gpurun_out/t_tile.log | head -80; exit 1; }
grep -E "PASS|FAIL" gpurun_out/t_tile.log | tail -50
timeout -k 10 300 python -u tools/engine_ab.py --out gpurun_out/r02_engine_ab.json > gpurun_out/engine_ab.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/engine_ab.log; exit 1; }
cat gpurun_out/engine_ab.log | grep '^{'
