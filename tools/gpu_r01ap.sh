set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/resolve_prof.py 10 16 > gpurun_out/resolve_prof.log 2>&1
