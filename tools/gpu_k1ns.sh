#!/bin/bash
# K1 chains per lane (TSG_K1_NS=2/3/4), kernel-only timing.  usage: tools/gpu_k1ns.sh TAG
set -o pipefail
out=gpurun_out/${1:-k1ns}
mkdir -p $out
for n in 2 3 4; do
  TSG_K1_NS=$n timeout -k 10 200 python -u tools/kab.py 1024 7 > $out/kab_ns$n.json 2> $out/kab_ns$n.err || { tail -5 $out/kab_ns$n.err; exit 1; }
  echo "ns=$n $(cat $out/kab_ns$n.json)"
done
