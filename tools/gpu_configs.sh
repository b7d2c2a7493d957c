#!/bin/bash
# BASELINE configs beyond configs[1] on one MI355X: new GPU tests, configs[0] end to end,
# configs[3] and configs[4] benches.  usage: tools/gpu_configs.sh TAG
set -o pipefail
tag=${1:-r2}
out=gpurun_out/$tag
mkdir -p $out
echo "== tests" && timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "config0 or layer" > $out/gpu_tests.log 2>&1 || { tail -20 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
echo "== configs[0]" && timeout -k 10 400 python -u tools/fs_bench.py > $out/fs_bench.json 2> $out/fs_bench.err || { tail -20 $out/fs_bench.err; exit 2; }
cat $out/fs_bench.json
echo "== configs[3]" && timeout -k 10 500 python -u bench.py --rules user1000 --steps 2 --warmup 1 --cpu-mib 32 > $out/bench_user1000.json 2> $out/bench_user1000.err || { tail -20 $out/bench_user1000.err; exit 3; }
cat $out/bench_user1000.json
echo "== configs[4]" && timeout -k 10 400 python -u bench.py --rules allow-exclude --steps 2 --warmup 1 --cpu-mib 256 > $out/bench_allow.json 2> $out/bench_allow.err || { tail -20 $out/bench_allow.err; exit 4; }
cat $out/bench_allow.json
echo done
