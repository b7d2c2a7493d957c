set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof6
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6/ks -o ks --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof6/ks.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof6/pf -o pf --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof6/pf.log 2>&1
