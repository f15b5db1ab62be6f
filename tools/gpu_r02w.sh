# sharded optimizer: GPU DP test (gloo, 2 ranks on one GPU) + N=2 rehearsal of both schedules
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -q -x --timeout 300 --timeout-method thread > gpurun_out/t_w.log 2>&1 || { echo T_FAILED; grep -E "FAIL|Error|assert" gpurun_out/t_w.log | head -40; exit 1; }
tail -1 gpurun_out/t_w.log
for o in sharded replicated; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --all-ranks-on-device0 --optimizer $o > gpurun_out/dp2_$o.log 2>&1 || { echo DP_FAILED; tail -30 gpurun_out/dp2_$o.log; exit 1; }
grep '^{' gpurun_out/dp2_$o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$o', d['value'], d['final_loss'], d['config']['parallelism'])"
done
