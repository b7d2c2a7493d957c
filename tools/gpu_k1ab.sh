#!/bin/bash
# K1 A/B on the GPU box: kernel-only timing per library variant (tools/build_variants.sh),
# then one SQ pass (instruction mix, LDS conflicts, waits) per variant named in SQ="...".
# usage: SQ="default legacy" tools/gpu_k1ab.sh TAG v1 v2 ...
set -o pipefail
tag=${1:-k1ab}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in default "$@"; do
  if [ "$v" = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 200 python -u tools/kab.py 1024 7 > $out/kab_$v.json 2> $out/kab_$v.err || { tail -5 $out/kab_$v.err; exit 1; }
  cat $out/kab_$v.json
done
for v in $SQ; do
  if [ "$v" = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  echo "== SQ $v"
  timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY \
    --output-format csv -d $out/sq_$v -o run -- python tools/kab.py 1024 3 > $out/sq_$v.log 2>&1 || { tail -5 $out/sq_$v.log; exit 2; }
done
unset TSG_LIB_VARIANT
echo done
