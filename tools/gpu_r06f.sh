#!/bin/bash
# Round 6: K1F staggered wave starts -- the K1F device tests on the default build (stagger 1),
# then kernel-only timing of the default and the fs0 (none) / fs2 (graded) variants.
set -o pipefail
out=gpurun_out/r06/${1:-f}
mkdir -p $out
echo "== k1f tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "k1_matches or k1f_ or adaptation or corpus_vs" > $out/k1f_tests.log 2>&1 || { tail -30 $out/k1f_tests.log; exit 1; }
tail -1 $out/k1f_tests.log
for rep in 1 2 3; do
for v in default fs0 fs2; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_${v}_$rep.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print(d['k1_ms'], d['k1_clk_ms'], d['gate_ms'], d['k2_ms'], d['chain_clk_ms'])")
done
done
echo done
