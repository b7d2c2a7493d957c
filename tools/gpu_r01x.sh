set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/k1sweep.py 4 ns2 > gpurun_out/k1sweep.log 2>&1
TSG_K1_NS=4 timeout -k 10 300 python -u tools/k1sweep.py 4 ns4 >> gpurun_out/k1sweep.log 2>&1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
