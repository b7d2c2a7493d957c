#!/bin/bash
# Kernel-only timing of library variants (tools/kab.py; variants built by
# tools/k1f_variants_build.sh or by hand).  usage: tools/gpu_kab_variants.sh TAG VARIANT...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_$v.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 1; }
  echo $v $(python -c "import json; d=json.load(open('$out/kab_$v.json')); print(d['k1_ms'], d['k1_GBps'], d['k1f_listed'])")
done
echo done
