#!/bin/bash
# Round 6: K1F on configs[3] (the never-matching literal slots leave K1F's literal count at
# 121): the config GPU tests, K1 matches, kernel-only timing of K1F + K1X against the
# automaton + K1X (knob k1_automaton=1), and the configs[3] bench line.
set -o pipefail
out=gpurun_out/r06/${1:-j3}
mkdir -p $out
echo "== tests" && timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  tests/test_gpu.py -k "user or k1_matches or k1f_ or adaptation or corpus_vs" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  timeout -k 10 240 python -u tools/kab.py 1024 5 --rules user1000 > $out/kab_k1f_$rep.json 2> $out/kab.err || { tail $out/kab.err; exit 2; }
  timeout -k 10 240 python -u tools/kab.py 1024 5 --rules user1000 --knob k1_automaton=1 > $out/kab_auto_$rep.json 2> $out/kab.err || { tail $out/kab.err; exit 2; }
  for v in k1f auto; do echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print({k: d[k] for k in ('k1_ms','gate_ms','k2_ms','k1_clk_ms','chain_clk_ms','k1f_listed','k1f_arrivals','k1_hot','k1x_records') if k in d})"); done
done
echo "== bench user1000" && timeout -k 10 400 python -u bench.py --rules user1000 --steps 3 --warmup 1 > $out/bench_u1000.json 2> $out/bench.err || { tail $out/bench.err; exit 3; }
python -c "import json; d=json.load(open('$out/bench_u1000.json')); r=d['roofline']; k=d['kernels']; print(d['value'], r['kernel'], r['frac'], k['k1_ms_per_batch'], k['gates_ms_per_batch'], k['k2_ms_per_batch'], r['chain_clock_ms_per_batch'])"
echo done
