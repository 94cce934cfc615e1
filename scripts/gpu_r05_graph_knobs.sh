#!/bin/bash
# hipGraph decode at TP = 1 vs eager, with the HIP runtime's graph knobs (packet capture, graph queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/gk
: > gpurun_out/gk/ab.jsonl
run() {  # name env... -- args
  local name=$1; shift
  ( env "$@" timeout -k 10 300 python bench.py --steps 200 --warmup 20 $GARGS > gpurun_out/gk/$name.log 2>&1 ) || { echo "$name failed"; tail -20 gpurun_out/gk/$name.log; exit 1; }
  tail -1 gpurun_out/gk/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'variant': '$name', 'value': d['value'], 'ms': d['ms_per_step'], 'host': d.get('host_ms_per_step'), 'graphs': d.get('graph_stats')}))" | tee -a gpurun_out/gk/ab.jsonl
}
for i in 1 2; do
  GARGS="" run eager$i KAFKA_X=0 || exit 1
  GARGS="--graphs" run graphs$i KAFKA_X=0 || exit 1
  GARGS="--graphs" run graphs_nopc$i DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
  GARGS="--graphs" run graphs_noq$i DEBUG_HIP_FORCE_GRAPH_QUEUES=0 || exit 1
done
