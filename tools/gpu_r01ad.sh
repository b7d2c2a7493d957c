set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "corpus_vs_cpu or custom or reference_cases_one" > gpurun_out/gpu_tests.log 2>&1
for d in 2 3 4; do
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --depth $d > gpurun_out/bench_d$d.log 2>&1
done
