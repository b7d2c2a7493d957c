#!/bin/bash
# Ingest / e2e / configs[4] check on the GPU box.  usage: tools/gpu_ingest.sh TAG
set -o pipefail
tag=${1:-ing}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== e2e fs" && timeout -k 10 300 python -u bench.py --e2e fs --steps 3 > $out/e2e_fs.json 2> $out/e2e_fs.err || { tail $out/e2e_fs.err; exit 2; }
cat $out/e2e_fs.json
echo "== e2e layer" && timeout -k 10 400 python -u bench.py --e2e layer --steps 3 > $out/e2e_layer.json 2> $out/e2e_layer.err || { tail $out/e2e_layer.err; exit 3; }
cat $out/e2e_layer.json
echo "== configs[4]" && timeout -k 10 400 python -u bench.py --rules allow-exclude --steps 2 --warmup 1 --cpu-mib 256 > $out/bench_allow.json 2> $out/bench_allow.err || { tail $out/bench_allow.err; exit 4; }
cat $out/bench_allow.json
echo done
