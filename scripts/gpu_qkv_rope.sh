set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "qkv_rope or rope_kv" -x -v --timeout 120 --timeout-method thread > gpurun_out/t_rope.log 2>&1 || { tail -40 gpurun_out/t_rope.log; exit 1; }
tail -3 gpurun_out/t_rope.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
ARMS="KAFKA_FUSE_QKV_ROPE=0;KAFKA_FUSE_QKV_ROPE=1" ROUNDS=2 STEPS=200 WARM=20 bash scripts/gpu_ab_env.sh
