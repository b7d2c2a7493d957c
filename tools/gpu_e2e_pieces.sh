#!/bin/bash
# e2e fs / layer at several piece floors (bench.py --piece-mib).  usage: tools/gpu_e2e_pieces.sh TAG MIB...
set -o pipefail
tag=${1:-e2ep}; shift
out=gpurun_out/$tag
mkdir -p $out
export TSG_LAYER_PROF=1
for m in "$@"; do
  for k in fs layer; do
    timeout -k 10 300 python -u bench.py --e2e $k --piece-mib $m --steps 3 > $out/${k}_$m.json 2> $out/${k}_$m.err || { tail $out/${k}_$m.err; exit 2; }
    echo "$k floor=$m $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" $out/${k}_$m.json)"
    grep -E "^(pieces)" $out/${k}_$m.err | tail -1
  done
done
echo done
