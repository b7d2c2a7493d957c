set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_walker.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_walker.log 2>&1
