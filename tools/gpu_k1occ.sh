#!/bin/bash
# K1 occupancy knobs: TSG_K1_NOREP=2 (no replicated class table, two 640-thread blocks per
# CU) and TSG_K1_SEG (chunks per chain), kernel-only timing + parity under the best knob.
# usage: tools/gpu_k1occ.sh TAG
set -o pipefail
out=gpurun_out/${1:-k1occ}
mkdir -p $out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u tools/kab.py 1024 7 > $out/kab_$n.json 2> $out/kab_$n.err || { tail -5 $out/kab_$n.err; exit 1; }
  echo "$n $(python -c "import json; d=json.load(open('$out/kab_$n.json')); print(d['k1_ms'], d['k2_ms'], d['candidates'])")"
}
run default X=1
run norep2 TSG_K1_NOREP=2
run norep2_seg7 TSG_K1_NOREP=2 TSG_K1_SEG=7
run norep2_seg6 TSG_K1_NOREP=2 TSG_K1_SEG=6
run seg7 TSG_K1_SEG=7
TSG_K1_NOREP=2 TSG_K1_SEG=7 timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > $out/gpu_tests_norep2.log 2>&1 || { tail -20 $out/gpu_tests_norep2.log; exit 2; }
tail -1 $out/gpu_tests_norep2.log
