set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 tools/kprof.py 1 2 > gpurun_out/prof/kt.log 2>&1
TSG_K1_DEBUG=1 timeout -k 10 300 python -u tools/kbench.py 1 256 > gpurun_out/kbench_noacc.log 2>&1
