#!/bin/bash
# Round 4 pass R: (1) tests — early-launch equality, wstream, tile attention with the 4-wave / 64-row variant (HALF:
# per-half softmax, VALU row sums, no spills); (2) tile anatomy 8 vs 4 waves; (3) bench 38aea4b (ab_older/) vs
# 3800543 (ab_old/) vs this tree vs this tree with 4-wave tiles, interleaved x2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
PYTHONPATH=$R timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "early or wstream or attn" > gpurun_out/t_r.log 2>&1 || { tail -40 gpurun_out/t_r.log; exit 1; }
tail -1 gpurun_out/t_r.log
KAFKA_TILE_WAVES=4 PYTHONPATH=$R timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "attn" > gpurun_out/t_r4.log 2>&1 || { tail -40 gpurun_out/t_r4.log; exit 1; }
echo "4-wave tiles: $(tail -1 gpurun_out/t_r4.log)"
for w in 8 4; do
  KAFKA_TILE_WAVES=$w PYTHONPATH=$R timeout -k 10 200 python -u benchmarks/attn_tile_anatomy.py --variants 3 --keys 576,2304 2>&1 | grep keys_per | sed "s/^/waves$w /" || exit 1
done
: > gpurun_out/bench_r.jsonl
for round in 1 2; do
for v in older new new4; do
  P=$R; E=""; [[ $v == old ]] && P=$R/ab_old; [[ $v == older ]] && P=$R/ab_older; [[ $v == new4 ]] && E="KAFKA_TILE_WAVES=4"
  (cd $P && env $E PYTHONPATH=$P timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $R/gpurun_out/bench_$v.log 2>&1) || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/bench_r.jsonl
  echo "$v $(tail -1 gpurun_out/bench_$v.log | cut -c100-175)"
done
done
