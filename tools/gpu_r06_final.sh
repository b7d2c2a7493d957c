#!/bin/bash
# Round 6 closing evidence: the GPU suite, smoke(), the default bench line, the same bench
# under rocprofv3 --kernel-trace (+ batch timeline), FETCH_SIZE and SQ passes, the traffic
# record for profiles/pmc/.  Every GPU step under its own limit; stops at the first failure.
set -o pipefail
out=gpurun_out/r06/${1:-final}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
echo "== smoke" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 2; }
tail -3 $out/smoke.log
echo "== bench" && timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 3; }
python -c "import json; d=json.load(open('$out/bench.json')); r=d['roofline']; k=d['kernels']; print(d['value'], 'ev', r['frac_events'], 'clk', r['frac_clock'], r['k1_clock_ms_per_batch'], k['k1_ms_per_batch'], 'chain', r['chain_clock_ms_per_batch'], r['post_k1_clock_ms_per_batch'], r['device_frac'], d['cpu_baseline'])"
echo "== traced bench" && timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_traced.json 2> $out/bench_traced.err || { tail $out/bench_traced.err; exit 4; }
python -c "import json; d=json.load(open('$out/bench_traced.json')); r=d['roofline']; k=d['kernels']; print(d['value'], 'ev', r['frac_events'], 'clk', r['frac_clock'], r['k1_clock_ms_per_batch'], k['k1_ms_per_batch'])"
f=$(ls $out/trace/*/run_kernel_trace.csv 2>/dev/null || ls $out/trace/run_kernel_trace.csv)
python tools/ktimeline.py $f > $out/timeline.txt && tail -25 $out/timeline.txt
echo "== FETCH_SIZE" && timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_fetch.out 2>&1 || { tail $out/pmc_fetch.out; exit 5; }
echo "== SQ" && timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY --output-format csv -d $out/pmc_sq -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/pmc_sq.out 2>&1 || { tail $out/pmc_sq.out; exit 6; }
python tools/pmc_traffic.py --record builtin $out/pmc_fetch/run_counter_collection.csv $out/bench.json \
  profiles/r06/${1:-final}/bench_pmc_fetch.csv > $out/pmc_builtin.json || exit 7
cat $out/pmc_builtin.json
echo done
