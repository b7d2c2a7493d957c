#!/bin/bash
# K1F A/B on one box: the GPU K1 tests on the default build, then kernel-only timing
# (tools/kab.py) of the default build and of library variants.  usage: tools/gpu_k1f_ab.sh TAG VARIANT...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== k1f tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "k1_matches or k1f_ or adaptation or corpus_vs or slot_prefix" > $out/k1f_tests.log 2>&1 || { tail -40 $out/k1f_tests.log; exit 1; }
tail -1 $out/k1f_tests.log
for rep in 1; do
for v in default "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_${v}_$rep.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print(d['k1_ms'], d['k1_GBps'], d['gate_ms'], d['k2_ms'], d['k1f_listed'], d['k1f_arrivals'])")
done
done
echo done
