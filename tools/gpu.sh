# One parameterised GPU job (replaces the per-experiment scripts). Run on the GPU box:
#   gpurun -- bash tools/gpu.sh [OUT=name] step [step ...]
# Steps (each under its own time limit; the job stops at the first failing step):
#   tests[:<pytest args>]  GPU parity suite (default: all of tests -m gpu)
#   smoke                  __graft_entry__.smoke()
#   bench[:<bench args>]   bench.py (default args: none -> the driver's default run incl. CPU baseline)
#   prof[:<bench args>]    rocprofv3 --kernel-trace --stats of bench.py (-> $OUT/prof, top kernels)
#   pmc[:<groups file>]    PMC passes over a short bench (tools/gpu_pmc.sh) + HBM traffic summary;
#                          BENCH_EXTRA / PMC_FILTER pass through
#   spread                 tools/render_spread.py (render PSNR per seed pair)
#   profpy:<script> [args] rocprofv3 --kernel-trace --stats of a python tool (-> $OUT/profpyN)
#   py:<script> [args]     any python tool under tools/ (120 s budget unless PY_TIMEOUT)
# Output: gpurun_out/$OUT (default gpurun_out/job).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=job
if [[ "$1" == OUT=* ]]; then OUT="${1#OUT=}"; shift; fi
D=gpurun_out/$OUT
mkdir -p "$D"
n=0
for step in "$@"; do
  n=$((n + 1))
  name="${step%%:*}"
  arg=""
  [[ "$step" == *:* ]] && arg="${step#*:}"
  log="$D/$n-$name.log"
  echo "== step $n: $step" | tee -a "$D/steps.txt"
  case "$name" in
    tests)
      timeout -k 10 900 python -u -m pytest ${arg:-tests} -m gpu -q -rf --timeout 200 --timeout-method thread > "$log" 2>&1 \
        || { echo "TESTS_FAILED"; grep -E "^FAILED|Error" "$log" | head -20; tail -5 "$log"; exit 1; }
      tail -1 "$log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || { echo SMOKE_FAILED; tail -20 "$log"; exit 1; }
      tail -1 "$log" ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > "$log" 2>&1 || { echo BENCH_FAILED; tail -20 "$log"; exit 1; }
      grep '^{' "$log" | cut -c1-600 ;;
    prof)
      rm -rf "$D/prof$n"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/prof$n" -o run -- python3 bench.py --no-cpu-baseline $arg > "$log" 2>&1 \
        || { echo PROF_FAILED; tail -20 "$log"; exit 1; }
      python3 tools/prof_top.py "$D/prof$n" | head -12 ;;
    pmc)
      PMC_OUT="$D/pmc$n" timeout -k 10 900 bash tools/gpu_pmc.sh ${arg:-tools/pmc_groups.txt} > "$log" 2>&1 || { echo PMC_FAILED; tail -10 "$log"; exit 1; }
      tag=$(python3 bench.py --print-workload ${BENCH_EXTRA:-})
      python3 tools/pmc_traffic.py "$D/pmc$n" "$D/pmc$n.traffic.json" "$tag" | tail -12 || true ;;
    spread)
      timeout -k 10 600 python -u tools/render_spread.py "$D/render_spread.json" > "$log" 2>&1 || { echo SPREAD_FAILED; tail -20 "$log"; exit 1; }
      tail -25 "$log" ;;
    profpy)
      # rocprofv3 kernel stats of a python tool: profpy:<script> [args]
      rm -rf "$D/profpy$n"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/profpy$n" -o run -- python3 $arg > "$log" 2>&1 \
        || { echo PROFPY_FAILED; tail -20 "$log"; exit 1; }
      python3 tools/prof_top.py "$D/profpy$n" | head -12 ;;
    py)
      timeout -k 10 ${PY_TIMEOUT:-120} python -u $arg > "$log" 2>&1 || { echo "PY_FAILED $arg"; tail -20 "$log"; exit 1; }
      tail -${PY_TAIL:-15} "$log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo JOB_OK
