#!/bin/bash
# Kernel-only timing (tools/kab.py) of library variants on builtin and user1000 rules.
# usage: tools/gpu_kab_variants.sh TAG variant...   (default = the product build)
set -o pipefail
out=gpurun_out/${1:-kabv}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "$@"; do
  for rules in builtin user1000; do
    if [ "$v" = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
    timeout -k 10 200 python -u tools/kab.py 1024 7 --rules $rules > $out/kab_${v}_$rules.json 2> $out/kab_${v}_$rules.err || { tail -5 $out/kab_${v}_$rules.err; exit 1; }
    cut -c1-200 $out/kab_${v}_$rules.json
  done
done
