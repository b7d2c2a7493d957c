#!/bin/bash
# kernel-only timing (tools/kab.py) of the default build and library variants on one rule
# set.  usage: tools/gpu_kab_rules.sh TAG RULES VARIANT...
set -o pipefail
tag=$1; rules=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in default "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 5 --rules $rules > $out/kab_${v}_$rules.json 2> $out/kab_${v}_$rules.err || { echo "fail $v"; tail $out/kab_${v}_$rules.err; exit 2; }
  echo $rules $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rules.json')); print(d['k1_ms'], d['gate_ms'], d['k2_ms'], d['k2_entries'])")
done
echo done
