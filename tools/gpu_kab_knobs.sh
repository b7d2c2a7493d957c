#!/bin/bash
# kernel-only timing (tools/kab.py) of the default build under knob sets.
# usage: tools/gpu_kab_knobs.sh TAG "knob=v knob=v" ...   (one quoted set per run; "" = none)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for set in "$@"; do
  args=""; for kv in $set; do args="$args --knob $kv"; done
  timeout -k 10 240 python -u tools/kab.py 1024 5 $args > $out/kab_knobs_$i.json 2> $out/kab_knobs_$i.err || { echo "fail [$set]"; tail $out/kab_knobs_$i.err; exit 2; }
  echo "[$set]" $(python -c "import json; d=json.load(open('$out/kab_knobs_$i.json')); print(d['k1_ms'], d['gate_ms'], d['k2_ms'], d['dev_GBps'], d['k2_items'], d['k2_entries'])")
  i=$((i+1))
done
echo done
