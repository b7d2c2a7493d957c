set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K1SWEEP_BIG=1048576 timeout -k 10 300 python -u tools/k1sweep.py 4 2 > gpurun_out/k1sweep.log 2>&1
K1SWEEP_BIG=65536 timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
K1SWEEP_BIG=1048576 TSG_K1_DEBUG=1 timeout -k 10 300 python -u tools/k1sweep.py 4 2 >> gpurun_out/k1sweep.log 2>&1
