#!/bin/bash
# Round 6: the layout's block scans fused (two exchanges per tile of groups) -- the GPU suite,
# kernel-only timing on the builtin rules and on configs[3].
set -o pipefail
out=gpurun_out/r06/${1:-v}
mkdir -p $out
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_b_$rep.json 2> $out/kab.err || { tail $out/kab.err; exit 2; }
  timeout -k 10 240 python -u tools/kab.py 1024 5 --rules user1000 > $out/kab_u_$rep.json 2> $out/kab.err || { tail $out/kab.err; exit 2; }
  for v in b u; do echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print('k1', d['k1_ms'], 'gates', d['gate_ms'], 'k2', d['k2_ms'], 'chain', d['chain_clk_ms'], 'post', d['post_k1_clk_ms'])"); done
done
echo done
