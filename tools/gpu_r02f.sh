# round-2: fixture parity, DP schedules, full GPU suite, N=1 bench, N=2 strong-scaling rehearsal (gloo, one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fixtures.py tests/test_gpu_dp.py -v --timeout 200 --timeout-method thread -k "dp" > gpurun_out/t_fix.log 2>&1 || { echo FIX_FAILED; grep -E "PASS|FAIL|Error|assert" gpurun_out/t_fix.log | head -60; exit 1; }
grep -E "PASS|FAIL" gpurun_out/t_fix.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u bench.py > gpurun_out/bench_n1.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench_n1.log; exit 1; }
grep '^{' gpurun_out/bench_n1.log
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --all-ranks-on-device0 > gpurun_out/bench_n2_rehearsal.log 2>&1 || { echo REH_FAILED; tail -30 gpurun_out/bench_n2_rehearsal.log; exit 1; }
grep '^{' gpurun_out/bench_n2_rehearsal.log | cut -c1-600
