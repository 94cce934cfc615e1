#!/bin/bash
# Headline-bench A/B on one MI355X + a rocprofv3 kernel-stats run of the default configuration.
# Variants (one JSON line each in gpurun_out/ab.jsonl): default | blas (hipBLASLt decode GEMMs) | graphs | overlap.
# Stops at the first failure (no retries). Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_bench_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
ARGS=${AB_ARGS:-"--steps 150 --warmup 40"}
VARIANTS=${AB_VARIANTS:-"default blas graphs"}
run() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  env "$@" timeout -k 10 300 python bench.py $ARGS $EXTRA > gpurun_out/ab_$name.log 2>&1
  local rc=$?
  if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/ab_$name.log; then echo "GPU fault in $name"; exit 3; fi
  [[ $rc == 0 ]] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/ab_$name.log; exit 1; }
  tail -1 gpurun_out/ab_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$name'; print(json.dumps(d))" >> gpurun_out/ab.jsonl
  tail -1 gpurun_out/ab.jsonl | cut -c1-260
}
for v in $VARIANTS; do
  case $v in
    default) EXTRA="" run default KAFKA_DECODE_GEMM=auto ;;
    blas) EXTRA="" run blas KAFKA_DECODE_GEMM=blas ;;
    graphs) EXTRA="--graphs" run graphs KAFKA_DECODE_GEMM=auto ;;
    overlap) EXTRA="" run overlap KAFKA_ATTN_OVERLAP=1 ;;
    graphs_overlap) EXTRA="--graphs" run graphs_overlap KAFKA_ATTN_OVERLAP=1 ;;
  esac
done
if [[ -z $NO_PROF ]]; then
  echo "== prof $(date +%T)"
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 60 --warmup 20 $PROF_ARGS > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "prof failed"; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
  tail -1 "$GRAFT_REPO_ROOT/gpurun_out/prof.log" | cut -c1-200
fi
echo "== done $(date +%T)"
