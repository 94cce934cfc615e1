#!/bin/bash
# Round 4 pass P: early-launch equality test (gated instantiations), then 38aea4b (ab_older/, before the tile
# prologue reorder) vs 3800543 (ab_old/, before the gates) vs this tree, interleaved x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
PYTHONPATH=$R timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "early or wstream" > gpurun_out/t_early.log 2>&1 || { tail -40 gpurun_out/t_early.log; exit 1; }
tail -1 gpurun_out/t_early.log
: > gpurun_out/bench_p.jsonl
for v in older old new older old new older old new; do
  P=$R; [[ $v == old ]] && P=$R/ab_old; [[ $v == older ]] && P=$R/ab_older
  (cd $P && PYTHONPATH=$P timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $R/gpurun_out/bench_$v.log 2>&1) || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/bench_p.jsonl
  echo "$v $(tail -1 gpurun_out/bench_$v.log | cut -c100-175)"
done
