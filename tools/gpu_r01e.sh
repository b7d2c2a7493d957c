set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/kbench.py 1 256 > gpurun_out/kbench.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 tools/kprof.py 1 3 > gpurun_out/prof/kt.log 2>&1
