#!/bin/bash
# Round 6: K1F lab (table per SIMD half, staggered starts), the K2 / corpus device tests on the
# current code, kernel-only timing (tools/kab.py) twice.
set -o pipefail
out=gpurun_out/r06/${1:-e}
mkdir -p $out
echo "== lab" && timeout -k 10 200 tools/k1f_lab 11 > $out/lab.json 2>&1 || { cat $out/lab.json; exit 1; }
grep -E "V3_runs|V6|V7|V8|2x512|MHz" $out/lab.json
echo "== tests" && timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu.py tests/test_gpu_configs.py tests/test_gpu_oracle_fixtures.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 2; }
tail -1 $out/tests.log
for rep in 1 2; do
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_$rep.json 2> $out/kab.err || { tail $out/kab.err; exit 3; }
  echo $rep $(python -c "import json; d=json.load(open('$out/kab_$rep.json')); print('k1', d['k1_ms'], 'gates', d['gate_ms'], 'k2', d['k2_ms'], 'chain_clk', d['chain_clk_ms'], 'post', d['post_k1_clk_ms'])")
done
echo done
