# A/B of builds on one box: current tree vs sibling trees (round-1 worktree _r01wt, variants _v*wt),
# kernel stats of the headline bench for each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ${VARIANTS:-cur r01}; do
  d=$GRAFT_REPO_ROOT; [ $v != cur ] && d=$GRAFT_REPO_ROOT/_${v}wt
  rm -rf gpurun_out/ab_$v
  (cd $d && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_$v -o run -- python3 bench.py --steps 50 --warmup 10 ${EXTRA:-} > $GRAFT_REPO_ROOT/gpurun_out/ab_$v.log 2>&1) || { echo AB_FAILED $v; tail -20 gpurun_out/ab_$v.log; exit 1; }
  python3 tools/prof_top.py gpurun_out/ab_$v > gpurun_out/ab_$v.top; head -4 gpurun_out/ab_$v.top | cut -c1-110
  grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log
done
