#!/bin/bash
# K1X words per lane per round (library variants x1, x8; default 4), user1000 kernel-only
# timing, then the configs[3] GPU parity tests.  usage: tools/gpu_k1x.sh TAG
set -o pipefail
out=gpurun_out/${1:-k1x}
mkdir -p $out
for v in default x1 x8; do
  if [ "$v" = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/kab.py 1024 5 --rules user1000 > $out/kab_$v.json 2> $out/kab_$v.err || { tail -5 $out/kab_$v.err; exit 1; }
  echo "$v $(cat $out/kab_$v.json)"
done
unset TSG_LIB_VARIANT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "user1000 or k1x or configs" > $out/gpu_tests.log 2>&1 || { tail -20 $out/gpu_tests.log; exit 2; }
tail -1 $out/gpu_tests.log
