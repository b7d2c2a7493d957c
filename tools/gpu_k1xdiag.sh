#!/bin/bash
# K1X verify diagnosis: kernel-only timing of configs[3] with the xdiag variant (verify
# counters) and the default library, and a builtin trace (gates kernels).
set -o pipefail
out=gpurun_out/${1:-xdiag}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== xdiag" && TSG_LIB_VARIANT=xdiag timeout -k 10 300 python -u tools/kab.py 1024 5 --rules user1000 > $out/xdiag.json 2>&1 || { tail $out/xdiag.json; exit 2; }
tail -1 $out/xdiag.json
echo "== builtin trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tb -o run -- \
  python tools/kab.py 1024 5 > $out/tb.out 2>&1 || { tail $out/tb.out; exit 3; }
grep variant $out/tb.out
cut -d, -f1-7 $out/tb/run_kernel_stats.csv | cut -c1-150
echo "== user1000 trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tu -o run -- \
  python tools/kab.py 1024 5 --rules user1000 > $out/tu.out 2>&1 || { tail $out/tu.out; exit 4; }
grep variant $out/tu.out
cut -d, -f1-7 $out/tu/run_kernel_stats.csv | cut -c1-150
