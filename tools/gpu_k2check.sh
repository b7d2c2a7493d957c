#!/bin/bash
# K2 check on the GPU box: GPU tests, then per-entry traces (builtin, user1000) with the
# counter build, then kernel-only timing.  usage: tools/gpu_k2check.sh TAG
set -o pipefail
tag=${1:-k2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -2 $out/gpu_tests.log
for r in builtin user1000; do
  echo "== trace $r"
  TSG_LIB_VARIANT=k2ctr timeout -k 10 300 python -u tools/k2trace.py run $out/k2_$r 1024 --rules $r > $out/k2_$r.log 2>&1 || exit 2
  python tools/k2trace.py report $out/k2_$r > $out/k2_${r}_report.json || exit 2
  echo "== kab $r"
  timeout -k 10 300 python -u tools/kab.py 1024 5 --rules $r > $out/kab_$r.json 2> $out/kab_$r.err || exit 3
  cat $out/kab_$r.json
done
echo "== SQ builtin"
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS \
  --output-format csv -d $out/sq -o run -- python tools/kab.py 1024 3 > $out/kab_sq.log 2>&1 || exit 4
echo done
