#!/bin/bash
# Quick GPU check: the GPU parity suite, then the headline bench and its rocprofv3 kernel
# trace.  usage: tools/gpu_quick.sh TAG [bench args]   (every GPU step under its own limit)
set -o pipefail
tag=${1:-quick}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== bench" && timeout -k 10 400 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 2; }
tail -c 2500 $out/bench.json
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $out/trace -o run -- \
  python bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $out/trace.out 2>&1 || { tail $out/trace.out; exit 3; }
cat $out/trace/run_kernel_stats.csv 2>/dev/null | cut -c1-160
echo done
