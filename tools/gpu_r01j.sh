set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/k1sweep.py 4 2 > gpurun_out/k1sweep.log 2>&1
TSG_K1_GRID=4 timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
TSG_K1_GRID=16 timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
