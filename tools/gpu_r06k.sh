#!/bin/bash
# Round 6: K2 claims peek before their atomic -- the GPU suite, kernel-only timing of the
# default against k2peek0 (every claim an atomic), a traced bench (kernel durations).
set -o pipefail
out=gpurun_out/r06/${1:-k2p}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
[ -n "$SKIP_TESTS" ] || echo "== gpu suite" && [ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $out/tests.log
for rep in 1 2; do
for v in default "$@"; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_${v}_$rep.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print('k1', d['k1_ms'], 'gates', d['gate_ms'], 'k2', d['k2_ms'], 'chain', d['chain_clk_ms'], 'post', d['post_k1_clk_ms'])")
done
done
unset TSG_LIB_VARIANT
[ -n "$SKIP_TRACE" ] && { echo done; exit 0; }
echo "== traced bench" && timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bench_traced.json 2> $out/bench_traced.err || { tail $out/bench_traced.err; exit 4; }
head -12 $out/trace/run_kernel_stats.csv | cut -d, -f1-4
echo done
