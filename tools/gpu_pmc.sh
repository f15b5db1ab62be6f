# PMC passes over a short bench run (PMC_CMD: another python command line) (one rocprofv3 run per counter group, per the pool's rules)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=${PMC_OUT:-gpurun_out/pmc_run}
rm -rf $out; mkdir -p $out
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $out/pass$i -o run -- python3 ${PMC_CMD:-bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile ${BENCH_EXTRA:-}} > $out/pass$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $out/pass$i.log; exit 1; }
  f=$(find $out/pass$i -name '*counter_collection.csv' | head -1)
  echo "== pass $i: $grp"
  python3 tools/pmc_summary.py "$f" "${PMC_FILTER:-tcnn_amd}"
done < "${1:-tools/pmc_groups.txt}"
