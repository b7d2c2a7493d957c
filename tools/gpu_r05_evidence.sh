#!/bin/bash
# Round-5 evidence: the GPU suite, then configs[1] (builtin) bench with kernel trace, FETCH_SIZE
# and SQ passes (tools/gpu_bench_prof.sh), then tools/layer_bench.py (1 GiB layer, ranks
# 1/2/4/8 rank by rank).  usage: tools/gpu_r05_evidence.sh TAG
set -o pipefail
tag=${1:-r05/final}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
bash tools/gpu_bench_prof.sh $tag/bench || exit 2
echo "== layer bench" && timeout -k 10 500 python -u tools/layer_bench.py 1 3 > $out/layer_bench.json 2> $out/layer_bench.err || { tail $out/layer_bench.err; exit 3; }
echo done
