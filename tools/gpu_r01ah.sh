set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_walker.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_walker.log 2>&1
TSG_LAYER_PROF=1 timeout -k 10 400 python -u tools/layer_bench.py 1 3 > gpurun_out/layer_bench.json 2> gpurun_out/layer_bench.err
