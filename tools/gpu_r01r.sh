set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/k1sweep.py 4 2 > gpurun_out/k1sweep.log 2>&1
export TSG_K1_DEBUG=1
timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
for v in nolds coalnolds; do
TSG_LIB_VARIANT=$v timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
done
