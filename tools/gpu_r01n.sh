set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TSG_K1_NS=4 TSG_K1_DEBUG=1
timeout -k 10 300 python -u tools/k1sweep.py 4 2 > gpurun_out/k1sweep.log 2>&1
for v in noruns nocls notab nolds; do
TSG_LIB_VARIANT=$v timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
done
