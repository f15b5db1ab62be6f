# N=2 data-parallel code path rehearsed on one GPU (gloo all-reduce; never a measurement)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --all-ranks-on-device0 > gpurun_out/dp2.log 2>&1 || { echo DP_FAILED; tail -30 gpurun_out/dp2.log; exit 1; }
grep '^{' gpurun_out/dp2.log | cut -c1-300
