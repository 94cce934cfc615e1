#!/bin/bash
# kernel + HIP API trace of a short headline run (kept on the box), reduced to the step-gap anatomy
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -d /tmp/ht -o run --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 10 > "$R/gpurun_out/ht.log" 2>&1 || { tail -30 "$R/gpurun_out/ht.log"; exit 1; }
cd "$R" && python scripts/step_gap_anatomy.py /tmp/ht 24 > gpurun_out/step_gap_anatomy.txt 2>&1; cat gpurun_out/step_gap_anatomy.txt
