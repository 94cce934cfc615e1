#!/bin/bash
# HIP runtime dispatch knobs vs the step-start GPU idle gap (eager headline): packet batching and flushing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/ck
run() {  # name env
  local name=$1 envs=$2
  ( env $envs timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/ck/$name.log 2>&1 ) || { echo "$name failed"; tail -5 gpurun_out/ck/$name.log; return 1; }
  tail -1 gpurun_out/ck/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['host_ms_per_step'])"
}
for i in 1 2; do
  run base$i "KAFKA_X=0" || exit 1
  run batch1_$i "DEBUG_CLR_MAX_BATCH_SIZE=1" || exit 1
  run flush_$i "GPU_FLUSH_ON_EXECUTION=1" || exit 1
done
