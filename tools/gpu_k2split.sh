#!/bin/bash
# K2 LDS split check: GPU tests, kernel-only timing (builtin, user1000) with kernel traces.
set -o pipefail
out=gpurun_out/${1:-k2split}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for rules in builtin user1000; do
  echo "== $rules" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$rules -o run -- \
    python tools/kab.py 1024 5 --rules $rules > $out/$rules.out 2>&1 || { tail $out/$rules.out; exit 2; }
  grep variant $out/$rules.out | cut -c1-220
  grep -E "k2_" $out/$rules/run_kernel_stats.csv | cut -d, -f1-7
done
