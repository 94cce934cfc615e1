#!/bin/bash
# Round 4 pass AH: configuration sweep of the decode GEMM on the current kernel at 64 rows (the headline's decode).
set -o pipefail
cd "$GRAFT_REPO_ROOT/benchmarks"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT:$GRAFT_REPO_ROOT/benchmarks; mkdir -p ../gpurun_out
timeout -k 10 400 python -u wstream_sweep.py --M ${SWEEP_M:-64} --shapes 8b.qkv,8b.o,8b.down,8b.gate_up > ../gpurun_out/sweep_ah.jsonl 2> ../gpurun_out/sweep_ah.err || { tail -20 ../gpurun_out/sweep_ah.err; exit 1; }
python - <<'PY'
import json
rows=[json.loads(l) for l in open('../gpurun_out/sweep_ah.jsonl')]
for shape in sorted({r['shape'] for r in rows}):
    rs=sorted([r for r in rows if r['shape']==shape], key=lambda r: r['us']+r['reduce_us']*0)
    print(shape, [(r['mt'],r['kc'],r['kw'],r['S'],r['us']) for r in rs[:5]])
PY
