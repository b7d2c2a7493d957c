#!/bin/bash
# K1F variants on one box: the K1F device tests on the variants that change results paths
# (TESTED=...), then kernel-only timing (tools/kab.py) of the default build and every variant.
#   usage: tools/gpu_r06_kvar.sh TAG "TESTED VARIANTS" VARIANT...
set -o pipefail
tag=$1; shift
tested=$1; shift
out=gpurun_out/r06/$tag
mkdir -p $out
for v in $tested; do
  export TSG_LIB_VARIANT=$v
  echo "== k1f tests $v" && timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "k1_matches or k1f_ or adaptation or corpus_vs" > $out/tests_$v.log 2>&1 || { tail -30 $out/tests_$v.log; exit 1; }
  tail -1 $out/tests_$v.log
done
unset TSG_LIB_VARIANT
for rep in 1 2; do
for v in default "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_${v}_$rep.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print(d['k1_ms'], d['k1_clk_ms'], d['k1_GBps'], d['gate_ms'], d['k2_ms'], d['k1f_listed'], d['k1f_arrivals'])")
done
done
echo done
