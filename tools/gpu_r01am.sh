set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof10
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof10/kt -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof10/kt.log 2>&1
