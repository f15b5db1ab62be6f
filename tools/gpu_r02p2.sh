# kernel statistics of config_oneblob as-is on the tile engine
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/p2
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/prof_oneblob.py > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
python3 tools/prof_top.py $OUT/prof > $OUT/top.txt; head -12 $OUT/top.txt
echo P2_OK
