#!/bin/bash
# e2e fs / layer, three runs each (host noise between runs).  usage: tools/gpu_e2e_rep.sh TAG
set -o pipefail
out=gpurun_out/${1:-e2erep}
mkdir -p $out
for i in 1 2 3; do
  for k in fs layer; do
    timeout -k 10 300 python -u bench.py --e2e $k --steps 3 > $out/${k}_$i.json 2> $out/${k}_$i.err || { tail $out/${k}_$i.err; exit 2; }
    echo "$k run $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['unpipelined'])" $out/${k}_$i.json)"
  done
done
