set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/k1sweep.py 4 base > gpurun_out/k1sweep.log 2>&1
for v in b384 b512; do
TSG_LIB_VARIANT=$v timeout -k 10 300 python -u tools/k1sweep.py 4 $v >> gpurun_out/k1sweep.log 2>&1
done
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
