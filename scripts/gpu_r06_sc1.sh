#!/bin/bash
# Round 6: full GPU suite on the hazard-safe sc1 stores (+ the fp32 numerics test); the suite again with sc1 stores
# at the round-5 rejected sites (RMSNorm / RoPE outputs); same-box A/B of those sites (SC1_AB=1); smoke. Stops at the
# first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; O=gpurun_out/r06; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest_gpu_default.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_default.log; grep -E "engine max" $O/pytest_gpu_default.log; [[ $rc == 0 ]] || { grep -E "FAILED|Error" $O/pytest_gpu_default.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep -E "smoke" $O/smoke.log | cut -c1-200
KAFKA_SC1_NORM=1 KAFKA_SC1_ROPE=1 timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu_sc1_norm_rope.log 2>&1
rc=$?; tail -3 $O/pytest_gpu_sc1_norm_rope.log; [[ $rc == 0 ]] || { grep -E "^FAILED" $O/pytest_gpu_sc1_norm_rope.log | head -30; exit 0; }
[[ -n $SC1_AB ]] && AB_SETS="base:KAFKA_X=0 sc1:KAFKA_SC1_NORM=1,KAFKA_SC1_ROPE=1" AB_ROUNDS=2 AB_ARGS="--steps 150 --warmup 20" bash scripts/gpu_ab_env.sh
exit 0
