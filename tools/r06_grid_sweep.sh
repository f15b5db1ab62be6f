# r06: grid-backward work split sweep (TCNN_GRID_BWD_RANGES: entry ranges per hashed level; TCNN_GRID_BWD_CHUNKS:
# point chunks) on the plain training step at 2^15 / 2^16 / 2^17 / 2^18 points (tools/dp_floor.py plain, eager)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/r06_grid_sweep; mkdir -p $D
for rc in "0 0" "4 0" "8 0" "0 2" "0 8" "4 8"; do
  set -- $rc; R=$1; C=$2; tag=r${R}_c${C}
  for lb in 15 16 17 18; do
    ( [ $R != 0 ] && export TCNN_GRID_BWD_RANGES=$R; [ $C != 0 ] && export TCNN_GRID_BWD_CHUNKS=$C
      timeout -k 10 120 python3 tools/dp_floor.py --schedules plain --steps 300 --batch-log2 $lb --out $D/${tag}_$lb.json > $D/${tag}_$lb.log 2>&1 ) || { tail -5 $D/${tag}_$lb.log; exit 1; }
  done
  python3 -c "
import json
print('$tag', [(lb, round(json.load(open('$D/${tag}_%d.json' % lb))['rows'][0]['gpu_us_per_step'], 2)) for lb in (15, 16, 17, 18)])"
done
