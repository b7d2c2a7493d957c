set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_walker.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pin.json 2> gpurun_out/bench_pin.err
TSG_NO_PIN=1 timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_nopin.json 2> gpurun_out/bench_nopin.err
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pin2.json 2> gpurun_out/bench_pin2.err
