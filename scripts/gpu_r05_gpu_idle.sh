#!/bin/bash
# GPU time inside vs between step spans (timing events, no profiler), eager and hipGraph replay
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/idle
for i in 1 2; do
  for a in "" "--graphs"; do
    n=eager; [[ -n $a ]] && n=graphs
    timeout -k 10 300 python bench.py --steps 200 --warmup 20 $a > gpurun_out/idle/$n$i.log 2>&1 || { tail -20 gpurun_out/idle/$n$i.log; exit 1; }
    tail -1 gpurun_out/idle/$n$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n$i', d['value'], d['ms_per_step'], d['gpu_ms_per_step'], d['host_ms_per_step'])"
  done
done
