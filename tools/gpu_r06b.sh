#!/bin/bash
# Round 6: the K1F cost bisection (tools/k1f_lab) and the GPU tests that now read the oracle's
# committed results (tests/golden/oracle_small/) instead of running oracle/ on the box.
set -o pipefail
out=gpurun_out/r06/${1:-b}
mkdir -p $out
echo "== lab" && timeout -k 10 200 tools/k1f_lab 11 > $out/lab.json 2>&1 || { cat $out/lab.json; exit 1; }
cat $out/lab.json
echo "== sample tests" && timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu.py tests/test_gpu_configs.py tests/test_walker.py tests/test_multirank.py \
  -k "oracle or config0 or multi_two or slot_ingest or larger_than_slot or two_ranks_layer_gpu" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 2; }
tail -2 $out/tests.log
echo "== smoke" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 3; }
cat $out/smoke.log
echo done
