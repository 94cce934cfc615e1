#!/bin/bash
# kernel-argument placement vs hipGraph replay speed: eager / graphs with HIP_FORCE_DEV_KERNARG 0 and 1
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/ka
run() {  # name env args
  local name=$1 envs=$2 a=$3
  ( env $envs timeout -k 10 300 python bench.py --steps 200 --warmup 20 $a > gpurun_out/ka/$name.log 2>&1 ) || { echo "$name failed"; tail -5 gpurun_out/ka/$name.log; return 1; }
  tail -1 gpurun_out/ka/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['value'], d['ms_per_step'], d['gpu_ms_per_step'])"
}
for i in 1 2; do
  run eager$i "KAFKA_X=0" "" || exit 1
  run eager_dk1_$i "HIP_FORCE_DEV_KERNARG=1" "" || exit 1
  run graphs$i "KAFKA_X=0" "--graphs" || exit 1
  run graphs_dk0_$i "HIP_FORCE_DEV_KERNARG=0" "--graphs" || exit 1
done
