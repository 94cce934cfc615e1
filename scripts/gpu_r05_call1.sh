#!/bin/bash
# round-5 first measurement call: decode attention sweep + PMC, then the pruned tree vs the r04 snapshot (and graphs),
# the kernel-shape trace of the headline, and the GPU tests of the kernels + engine
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r05_decode_pmc.sh || exit 1
AB_PAIRS=2 AB_SEQ="new old newg" AB_TESTS="tests/test_kernels_gpu.py tests/test_engine_gpu.py" AB_PROF=1 bash scripts/gpu_r05_ab.sh
