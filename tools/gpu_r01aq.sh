set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/resolve_prof.py 10 16 > gpurun_out/resolve_prof.log 2>&1
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_nl.json 2> gpurun_out/bench_nl.err
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
