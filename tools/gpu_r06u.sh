#!/bin/bash
# Round 6: configs[3] gates -- config GPU tests, kernel-only user1000 timing of the default
# against g48 (the keyword -> group table in LDS only up to 48 KiB), a traced user1000 bench.
set -o pipefail
out=gpurun_out/r06/${1:-u3}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
for v in default ${VARIANTS:-g48}; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 5 --rules user1000 > $out/kab_${v}_$rep.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 2; }
  echo $rep $v $(python -c "import json; d=json.load(open('$out/kab_${v}_$rep.json')); print('k1', d['k1_ms'], 'gates', d['gate_ms'], 'k2', d['k2_ms'], 'chain', d['chain_clk_ms'])")
done
done
unset TSG_LIB_VARIANT
echo "== traced" && timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python -u bench.py --rules user1000 --steps 2 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 3; }
head -16 $out/trace/run_kernel_stats.csv | cut -d, -f1-4
echo done
