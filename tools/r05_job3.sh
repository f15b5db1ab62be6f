# r05: full GPU suite, tile A/B, 8-rank peer-exchange bench rehearsal on one GPU (configs[4] shard sizes)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r05_j3}; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 200 python3 tools/tile_ts_ab.py > $D/ab64.log 2>&1 || { tail -5 $D/ab64.log; exit 1; }
grep '^{' $D/ab64.log | cut -c1-150
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 8 --steps 20 --warmup 5 --dist-backend gloo --all-ranks-on-device0 --no-cpu-baseline > $D/dp8.log 2>&1 || { echo DP8_FAILED; tail -30 $D/dp8.log; exit 1; }
grep '^{' $D/dp8.log | cut -c1-400
