#!/bin/bash
# K1 kernel-only timing per library variant (tools/build_variants.sh).  usage: tools/gpu_k1var.sh TAG v1 v2 ...
set -o pipefail
tag=${1:-k1v}; shift
out=gpurun_out/$tag
mkdir -p $out
for v in default "$@"; do
  if [ "$v" = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/kab.py 1024 7 > $out/kab_$v.json 2> $out/kab_$v.err || { tail -5 $out/kab_$v.err; exit 1; }
  cat $out/kab_$v.json
done
