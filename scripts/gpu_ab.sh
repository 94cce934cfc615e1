#!/bin/bash
# A/B of the opt-in engine features on one MI355X (headline bench workload, shorter run):
#   base | hipGraph decode (--graphs) | cascade/suffix stream overlap (KAFKA_ATTN_OVERLAP=1) | both
# One JSON line per variant in gpurun_out/ab.jsonl. Each variant runs under its own timeout; the script stops at
# the first failure (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
ARGS=${AB_ARGS:-"--steps 150 --warmup 40"}
run() {
  local name=$1; shift
  echo "== $name"
  env "$@" timeout -k 10 400 python bench.py $ARGS ${EXTRA} > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }
  tail -1 gpurun_out/ab_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$name'; print(json.dumps(d))" >> gpurun_out/ab.jsonl
  tail -1 gpurun_out/ab.jsonl | cut -c1-220
}
EXTRA="" run base KAFKA_ATTN_OVERLAP=0
EXTRA="--graphs" run graphs KAFKA_ATTN_OVERLAP=0
EXTRA="" run overlap KAFKA_ATTN_OVERLAP=1
EXTRA="--graphs" run graphs_overlap KAFKA_ATTN_OVERLAP=1
