#!/bin/bash
# The whole GPU suite, then kernel-only timing (tools/kab.py) of the default build and of
# library variants.  usage: tools/gpu_check.sh TAG [VARIANT...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for v in default "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_$v.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $v $(python -c "import json; d=json.load(open('$out/kab_$v.json')); print(d['k1_ms'], d['k1_GBps'], d['gate_ms'], d['k2_ms'], d['dev_GBps'], d['k1f_listed'], d['k1f_arrivals'])")
done
if [ -n "$KAB_RULES" ]; then
  for r in $KAB_RULES; do
    unset TSG_LIB_VARIANT
    timeout -k 10 240 python -u tools/kab.py 1024 5 --rules $r > $out/kab_default_$r.json 2> $out/kab_$r.err || { echo "fail $r"; tail $out/kab_$r.err; exit 3; }
    echo $r $(python -c "import json; d=json.load(open('$out/kab_default_$r.json')); print(d['k1_ms'], d['gate_ms'], d['k2_ms'], d['dev_GBps'])")
  done
fi
echo done
