#!/bin/bash
# GPU parity suite on the box: one pytest process, every test under a thread timeout.
# usage: tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
K=${2:+-k "$2"}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread $K \
  > gpurun_out/gpu_tests_$tag.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests_$tag.log
exit $rc
