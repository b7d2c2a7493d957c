#!/bin/bash
# FETCH_SIZE calibration for K1's access pattern + a one-step device timeline (kernels and
# memory copies) of the bench.  usage: tools/gpu_calib_timeline.sh TAG [bench args]
set -o pipefail
tag=${1:-r2}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== calib timing" && timeout -k 10 120 tools/fetch_calib > $out/calib_timing.txt 2>&1 || exit 1
cat $out/calib_timing.txt
echo "== calib FETCH_SIZE" && timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/calib -o calib -- tools/fetch_calib > $out/calib.out 2>&1 || exit 2
echo "== timeline" && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/timeline -o run -- \
  python bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $out/timeline.out 2>&1 || exit 3
find $out -name "*.csv"
echo done
