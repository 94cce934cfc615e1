cd "$GRAFT_REPO_ROOT"
KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 500 python benchmarks/skinny_bench.py > gpurun_out/skinny_vs2.jsonl 2>&1 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/skinny_vs2.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["gemm"], d["M"], "blas", d["hipblaslt_us"], "skinny", d["skinny_us"], "mt8", d["mt8_us"])
PY
