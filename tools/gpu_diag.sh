#!/bin/bash
# Kernel diagnosis on the GPU box: K2 per-entry traces (builtin, user1000) and K1 SQ LDS
# counters per library variant (tools/build_variants.sh).  usage: tools/gpu_diag.sh TAG [variants]
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -o pipefail
tag=${1:-diag}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== k2 trace builtin"
timeout -k 10 300 python -u tools/k2trace.py run $out/k2b 1024 > $out/k2b.log 2>&1 || exit 1
python tools/k2trace.py report $out/k2b > $out/k2b_report.json || exit 1
echo "== k2 trace user1000"
timeout -k 10 300 python -u tools/k2trace.py run $out/k2u 1024 --rules user1000 > $out/k2u.log 2>&1 || exit 2
python tools/k2trace.py report $out/k2u > $out/k2u_report.json || exit 2
for v in default "$@"; do
  echo "== SQ $v"
  if [ "$v" = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS \
    --output-format csv -d $out/sq_$v -o run -- python tools/kab.py 1024 3 > $out/kab_$v.log 2>&1 || exit 3
  tail -1 $out/kab_$v.log
done
unset TSG_LIB_VARIANT
echo done
