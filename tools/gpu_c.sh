#!/bin/bash
# GPU tests + K2 entry trace + bench/rocprof evidence.  usage: tools/gpu_c.sh TAG
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== k2 trace" && timeout -k 10 300 python -u tools/k2trace.py run $out/k2 > $out/k2trace.out 2>&1 || { tail $out/k2trace.out; exit 2; }
tools/gpu_bench_prof.sh $tag || exit 3
echo done
