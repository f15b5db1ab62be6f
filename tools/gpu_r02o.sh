# which earlier parity test makes test_inference_matches_oracle fail
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in "grid_forward_bit_exact or inference" "trainer_init or inference" "fused_step or inference" "adam_step or inference" "inference"; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "$k" --timeout 100 --timeout-method thread > gpurun_out/t_o.log 2>&1; rc=$?
  echo "[$k] rc=$rc $(tail -1 gpurun_out/t_o.log)"
  [ $rc -gt 1 ] && exit 1
done
exit 0
