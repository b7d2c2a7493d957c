#!/bin/bash
# Round 6: K1F with per-block dynamic chunks -- K1F device tests, kernel-only timing, the
# per-wave trace.
set -o pipefail
out=gpurun_out/r06/${1:-h}
mkdir -p $out
echo "== k1f tests" && timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "k1_matches or k1f_ or adaptation or corpus_vs or event_list" > $out/k1f_tests.log 2>&1 || { tail -30 $out/k1f_tests.log; exit 1; }
tail -1 $out/k1f_tests.log
for rep in 1 2; do
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_$rep.json 2> $out/kab.err || { tail $out/kab.err; exit 2; }
  echo $rep $(python -c "import json; d=json.load(open('$out/kab_$rep.json')); print('k1', d['k1_ms'], d['k1_clk_ms'], 'gates', d['gate_ms'], 'k2', d['k2_ms'], 'chain_clk', d['chain_clk_ms'])")
done
timeout -k 10 240 python tools/k1ftrace.py run $out 1024 > $out/trace_run.log 2>&1 && python tools/k1ftrace.py report $out > $out/k1ftrace_report.json && python -c "import json; d=json.load(open('$out/k1ftrace_report.json')); print('span', d['span_us'], 'dur', d['dur_us_q'], 'end', d['end_us_q'], 'tiles', d['tiles_q'])"
echo done
