# r06: hipGraph replay vs eager of the training step (tools/dp_floor.py plain) under the HIP runtime's
# graph switches (DEBUG_CLR_GRAPH_PACKET_CAPTURE, DEBUG_HIP_GRAPH_BATCH_SIZE, DEBUG_HIP_FORCE_GRAPH_QUEUES)
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; D=gpurun_out/r06_graph_env; mkdir -p $D
run() {  # $1 tag, rest env assignments
  tag=$1; shift
  for lb in 15 18; do
    env "$@" timeout -k 10 200 python3 tools/dp_floor.py --schedules plain --steps 400 --batch-log2 $lb --out $D/${tag}_$lb.json > $D/${tag}_$lb.log 2>&1 || { tail -5 $D/${tag}_$lb.log; return 1; }
    python3 -c "import json; d=json.load(open('$D/${tag}_$lb.json')); print('$tag', $lb, [(r['schedule'], round(r['gpu_us_per_step'],2), round(r['host_issue_us_per_step'],2)) for r in d['rows']])"
  done
}
run default X=1 && run capture0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run capture1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && \
run batch1 DEBUG_HIP_GRAPH_BATCH_SIZE=1 && run batch64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 && run queues0 DEBUG_HIP_FORCE_GRAPH_QUEUES=0 && \
run queues1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
