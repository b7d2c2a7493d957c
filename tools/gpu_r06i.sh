#!/bin/bash
# Round 6: K1F reserve chunks (K1F_STEAL) -- K1F device tests, kernel-only timing of the
# default and the variants named on the command line, per-wave traces (ftr: default with the
# trace, ftr0: slot shares only).
set -o pipefail
out=gpurun_out/r06/${1:-i}; shift
mkdir -p $out
echo "== k1f tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "k1_matches or k1f_ or adaptation or corpus_vs or event_list" > $out/k1f_tests.log 2>&1 || { tail -30 $out/k1f_tests.log; exit 1; }
tail -1 $out/k1f_tests.log
for rep in 1 2; do
for v in default "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_${v}_$rep.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print('k1', d['k1_ms'], d['k1_clk_ms'], 'chain', d['chain_clk_ms'])")
done
done
for v in ftr ftr0; do
  export TSG_LIB_VARIANT=$v
  mkdir -p $out/$v
  timeout -k 10 240 python tools/k1ftrace.py run $out/$v 1024 > $out/$v/run.log 2>&1 || { tail $out/$v/run.log; exit 3; }
  python tools/k1ftrace.py report $out/$v > $out/$v/report.json && python -c "import json; d=json.load(open('$out/$v/report.json')); print('$v span', d['span_us'], 'end', d['end_us_q'], d['by_slot'])"
done
echo done
