set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 12 14 15 16 20; do
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --host-threads $t > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t$t.err
done
