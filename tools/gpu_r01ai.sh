set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_stride.json 2> gpurun_out/bench_stride.err
TSG_K1_STRIDE=0 timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_nostride.json 2> gpurun_out/bench_nostride.err
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_stride2.json 2> gpurun_out/bench_stride2.err
