set -o pipefail
cd $GRAFT_REPO_ROOT
export KAFKA_NO_BUILD=1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/kt1.log 2>&1
echo "exit $?" >> gpurun_out/kt1.log
tail -30 gpurun_out/kt1.log
