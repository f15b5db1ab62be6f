# r06 start of round: default bench, rocprof breakdown of the per-rank step at 2^15 (plain and peer on one
# rank), and the peer step of 8 ranks time-sharing one GPU (each rank under its own rocprofv3, started by
# this shell -- no process that touched the GPU launches another)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/${OUT:-r06_base}; mkdir -p $D
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | cut -c1-200
for s in plain peer; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$s -o run -- python3 tools/dp_floor.py --schedules $s --steps 400 --batch-log2 ${LOG2B:-15} --out $D/floor_$s.json > $D/prof_$s.log 2>&1 || { tail -5 $D/prof_$s.log; exit 1; }
  f=$(find $D/prof_$s -name '*kernel_stats.csv' | head -1); cp "$f" $D/kstats_$s.csv; cut -d, -f1-4 "$f" | head -9 | cut -c1-90
  python3 -c "import json; d=json.load(open('$D/floor_$s.json')); [print(r['schedule'], round(r['gpu_us_per_step'],2), round(r['host_issue_us_per_step'],2)) for r in d['rows']]"
done
if [ -n "$R8" ]; then
  port=$((29500 + RANDOM % 1000)); pids=""
  for r in 0 1 2 3 4 5 6 7; do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=8 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof8_r$r -o run -- python3 bench.py --gpus 8 --all-ranks-on-device0 --dist-backend gloo --steps 100 --warmup 10 --no-profile > $D/r8_$r.log 2>&1 &
    pids="$pids $!"
  done
  rc=0; for p in $pids; do wait $p || rc=1; done
  [ $rc -eq 0 ] || { tail -5 $D/r8_0.log; exit 1; }
  grep '^{' $D/r8_0.log | cut -c1-200
  f=$(find $D/prof8_r0 -name '*kernel_stats.csv' | head -1); cp "$f" $D/kstats_8rank_r0.csv; cut -d, -f1-4 "$f" | head -9 | cut -c1-90
fi
