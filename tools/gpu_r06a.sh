#!/bin/bash
# Round 6 first GPU pass: the streaming floor microbenchmark, the K1F tests (with the new
# many-tiles-per-wave test), kernel-only timing with the in-kernel clocks, a short bench line.
set -o pipefail
out=gpurun_out/r06/${1:-a}
mkdir -p $out
echo "== stream floor" && timeout -k 10 150 tools/stream_floor 15 > $out/stream_floor.json 2>&1 || { cat $out/stream_floor.json; exit 1; }
cat $out/stream_floor.json
echo "== k1f tests" && timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "k1_matches or k1f_ or adaptation" > $out/k1f_tests.log 2>&1 || { tail -40 $out/k1f_tests.log; exit 2; }
tail -1 $out/k1f_tests.log
echo "== kab" && timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab.json 2> $out/kab.err || { tail $out/kab.err; exit 3; }
cat $out/kab.json
echo "== bench" && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 4; }
python -c "import json; d=json.load(open('$out/bench.json')); r=d['roofline']; print(d['value'], r['frac_events'], r['frac_clock'], r['k1_clock_ms_per_batch'], d['kernels']['k1_ms_per_batch'], r['chain_clock_ms_per_batch'], r['k1_gates_k2_frac'], r['chain_frac_clock'])"
echo done
