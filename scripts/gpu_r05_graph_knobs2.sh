#!/bin/bash
# hipGraph replay vs eager with DEBUG_HIP_GRAPH_BATCH_SIZE (graph kernel packets written per submission batch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/gk2
run() {  # name env graphs-flag
  local name=$1 envs=$2 a=$3
  ( env $envs timeout -k 10 300 python bench.py --steps 200 --warmup 20 $a > gpurun_out/gk2/$name.log 2>&1 ) || { echo "$name failed"; tail -20 gpurun_out/gk2/$name.log; exit 1; }
  tail -1 gpurun_out/gk2/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d.get('graph_stats'))"
}
for i in 1 2; do
  run eager$i "KAFKA_X=0" "" || exit 1
  run graphs$i "KAFKA_X=0" "--graphs" || exit 1
  run graphs_b1k$i "DEBUG_HIP_GRAPH_BATCH_SIZE=1024" "--graphs" || exit 1
  run graphs_b8$i "DEBUG_HIP_GRAPH_BATCH_SIZE=8" "--graphs" || exit 1
done
