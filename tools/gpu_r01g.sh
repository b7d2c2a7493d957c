set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bk -o bk --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_prof.json 2> gpurun_out/prof/bench_prof.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pf -o pf --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench_pmc.json 2> gpurun_out/prof/bench_pmc.err
