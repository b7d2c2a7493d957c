#!/bin/bash
# Round 6: K1F cost bisection (tools/k1f_lab), the GPU tests on the oracle's committed results,
# smoke(), then the configs[1] bench line untraced and under rocprofv3 --kernel-trace (the
# same run's in-kernel clocks beside the trace's durations), and the batch timeline.
set -o pipefail
out=gpurun_out/r06/${1:-c}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== lab" && timeout -k 10 200 tools/k1f_lab 11 > $out/lab.json 2>&1 || { cat $out/lab.json; exit 1; }
cat $out/lab.json
echo "== k1f tests" && timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu.py -k "event_list or k1f_ or k1_matches" > $out/k1f_tests.log 2>&1 || { tail -40 $out/k1f_tests.log; exit 2; }
tail -1 $out/k1f_tests.log
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 2; }
tail -2 $out/tests.log
echo "== smoke" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 3; }
cat $out/smoke.log
echo "== bench" && timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 4; }
python -c "import json; d=json.load(open('$out/bench.json')); r=d['roofline']; k=d['kernels']; print(d['value'], 'ev', r['frac_events'], 'clk', r['frac_clock'], r['k1_clock_ms_per_batch'], k['k1_ms_per_batch'], 'chain', r['chain_clock_ms_per_batch'], r['k1_gates_k2_frac'], r['chain_frac_clock'], r['device_frac'])"
echo "== traced bench" && timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_traced.json 2> $out/bench_traced.err || { tail $out/bench_traced.err; exit 5; }
python -c "import json; d=json.load(open('$out/bench_traced.json')); r=d['roofline']; k=d['kernels']; print(d['value'], 'ev', r['frac_events'], 'clk', r['frac_clock'], r['k1_clock_ms_per_batch'], k['k1_ms_per_batch'])"
f=$(ls $out/trace/*/run_kernel_trace.csv 2>/dev/null || ls $out/trace/run_kernel_trace.csv)
python tools/ktimeline.py $f > $out/timeline.txt && cat $out/timeline.txt
echo done
