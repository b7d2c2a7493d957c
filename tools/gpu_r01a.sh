set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1 || true
(go version || echo nogo) > gpurun_out/go.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --gb 1 --steps 3 --warmup 1 > gpurun_out/bench1.log 2>&1
timeout -k 10 300 python -u tools/kbench.py 1 256 > gpurun_out/kbench.log 2>&1
