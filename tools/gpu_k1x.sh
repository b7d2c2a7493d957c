#!/bin/bash
# K1X (configs[3]) check: the user-rule GPU parity tests, then kernel-only timing and a
# rocprofv3 kernel trace per K1X window step.  usage: tools/gpu_k1x.sh TAG [steps...]
set -o pipefail
tag=${1:-k1x}; shift
steps=${@:-0 4 2 1}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for st in $steps; do
  kn=""; [ "$st" != 0 ] && kn="--knob x_step=$st"
  echo "== step $st" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/s$st -o run -- \
    python tools/kab.py 1024 5 --rules user1000 $kn > $out/s$st.out 2>&1 || { tail $out/s$st.out; exit 2; }
  tail -1 $out/s$st.out
  grep -E "k1_kernel|k1x" $out/s$st/run_kernel_stats.csv | cut -d, -f1-7
done
echo done
