set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/kbench.py 1 256 > gpurun_out/kbench.log 2>&1
TSG_K1_DEBUG=1 timeout -k 10 300 python -u tools/kbench.py 1 256 > gpurun_out/kbench_noacc.log 2>&1
