#!/bin/bash
# Round 6: K1F lab (block shapes of the no-copy queue), kernel-only A/B of K1F's event list
# (default) against the gates pass (no_k1f_list), and an SQ pass of the default.
set -o pipefail
out=gpurun_out/r06/${1:-d}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== lab" && timeout -k 10 200 tools/k1f_lab 11 > $out/lab.json 2>&1 || { cat $out/lab.json; exit 1; }
grep -E "V3_runs|V6|2x512|4x256|MHz" $out/lab.json
for rep in 1 2; do
  for kn in "" "--knob no_k1f_list=1"; do
    tag=$(echo "x$kn" | tr -cd 'a-z0-9')
    timeout -k 10 240 python -u tools/kab.py 1024 7 $kn > $out/kab_${tag}_$rep.json 2> $out/kab_$tag.err || { tail $out/kab_$tag.err; exit 2; }
    echo $rep $tag $(python -c "import json; d=json.load(open('$out/kab_${tag}_$rep.json')); print('k1', d['k1_ms'], 'gates', d['gate_ms'], 'k2', d['k2_ms'], 'chain_clk', d['chain_clk_ms'], 'post', d['post_k1_clk_ms'])")
  done
done
echo "== SQ" && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $out/pmc_sq -o run -- \
  python tools/kab.py 1024 3 > $out/pmc_sq.out 2>&1 || { tail $out/pmc_sq.out; exit 3; }
python tools/sq_summary.py $(ls $out/pmc_sq/*/run_counter_collection.csv $out/pmc_sq/run_counter_collection.csv 2>/dev/null | head -1) k1f --bytes 1073741824 > $out/sq_k1f.json; cat $out/sq_k1f.json | head -40
echo done
