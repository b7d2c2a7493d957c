#!/bin/bash
# Kernel trace of tools/kab.py (one seeded 1 GiB batch scanned repeatedly): per-kernel stats
# and the raw trace for the per-batch timeline (tools/ktimeline.py).  usage: tools/gpu_kprof.sh TAG [kab args]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python tools/kab.py 1024 3 "$@" > $out/kab.json 2> $out/trace.err || { tail $out/trace.err; exit 4; }
cat $out/kab.json
cut -c1-150 $out/trace/run_kernel_stats.csv | head -16
echo done
