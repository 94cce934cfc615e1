#!/bin/bash
# decode GEMM sweep with the 256-column (CT = 8) workgroups at 64..128 rows, plus the stream GEMM tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "wstream" > gpurun_out/call4_tests.log 2>&1 || { tail -30 gpurun_out/call4_tests.log; exit 1; }
tail -2 gpurun_out/call4_tests.log
cd benchmarks && timeout -k 10 600 python wstream_sweep.py --M 32,64,96,114,128 --shapes 8b.qkv,8b.o,8b.gate_up,8b.down > ../gpurun_out/wstream_sweep_ct8.jsonl 2>&1 || { tail -20 ../gpurun_out/wstream_sweep_ct8.jsonl; exit 1; }
python - <<'PY'
import json
rows=[json.loads(l) for l in open('../gpurun_out/wstream_sweep_ct8.jsonl') if l.startswith('{')]
by={}
for r in rows:
    by.setdefault((r['shape'],r['M']),[]).append((r['us']+r['reduce_us'],r))
for k,v in sorted(by.items()):
    v.sort(key=lambda x:x[0])
    print(k, ' | '.join(f"{t:.1f} mt{r['mt']} kc{r['kc']} kw{r['kw']} ct{r['ct']} pf{r['pf']} S{r['S']} e{r['err']}" for t,r in v[:5]))
PY
