#!/bin/bash
# K1X verify kernel parts: rocprofv3 kernel trace of configs[3] kernel-only timing per
# library variant (tools/build_variants.sh).  usage: tools/gpu_xv.sh TAG variant...
set -o pipefail
out=gpurun_out/${1:-xv}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "$@"; do
  echo "== $v" && TSG_LIB_VARIANT=$([ $v = default ] || echo $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run -- \
    python tools/kab.py 1024 5 --rules user1000 > $out/$v.out 2>&1 || { tail $out/$v.out; exit 2; }
  grep variant $out/$v.out
  grep -E "k1x|k2_dense" $out/$v/run_kernel_stats.csv | cut -d, -f1-7
done
