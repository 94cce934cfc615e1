#!/bin/bash
# host time per step (eager / graphs) + decode GEMM config sweep at 64..128 rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
for extra in "" "--graphs"; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 $extra > gpurun_out/host_ms$extra.log 2>&1 || { tail -20 gpurun_out/host_ms$extra.log; exit 1; }
  tail -1 gpurun_out/host_ms$extra.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$extra', d['value'], d['ms_per_step'], d['host_ms_per_step'], d['graph_stats'])"
done
cd benchmarks && timeout -k 10 600 python wstream_sweep.py --M 64,96,114,128 --shapes 8b.qkv,8b.o,8b.gate_up,8b.down > ../gpurun_out/wstream_sweep_r05.jsonl 2>&1 || { tail -20 ../gpurun_out/wstream_sweep_r05.jsonl; exit 1; }
python - <<'PY'
import json
rows=[json.loads(l) for l in open('../gpurun_out/wstream_sweep_r05.jsonl') if l.startswith('{')]
best={}
for r in rows:
    k=(r['shape'],r['M']); t=r['us']+r['reduce_us']
    if k not in best or t<best[k][0]: best[k]=(t,r)
for k,(t,r) in sorted(best.items()): print(k, round(t,1), {x:r[x] for x in ('mt','kc','kw','S','us','reduce_us')})
PY
