#!/bin/bash
# kernel traces of the headline eager and with --graphs (same box), for a per-kernel / gap comparison
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for m in eager graphs; do
  a=""; [[ $m == graphs ]] && a="--graphs"
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/gt_$m" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 $a > "$R/gpurun_out/gt_$m.log" 2>&1 || { tail -30 "$R/gpurun_out/gt_$m.log"; exit 1; }
done
echo done
