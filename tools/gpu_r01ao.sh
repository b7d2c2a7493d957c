set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof11
export TMPDIR=/tmp
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11/ks -o ks --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof11/ks.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof11/pf -o pf --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof11/pf.log 2>&1
