set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err
timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/bench_s40.json 2> gpurun_out/bench_s40.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --depth 6 > gpurun_out/bench_s20d6.json 2> gpurun_out/bench_s20d6.err
