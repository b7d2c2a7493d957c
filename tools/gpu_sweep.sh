#!/bin/bash
# A/B sweep of bench settings on the GPU box.
# usage: tools/gpu_sweep.sh TAG "ENV=V ...|bench args" ...   (first one also runs the GPU tests
# when GPU_TESTS=1)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
i=0
for cfg in "$@"; do
  i=$((i+1))
  echo "== $cfg"
  envs=${cfg%%|*}; bargs=${cfg#*|}; [ "$bargs" = "$cfg" ] && bargs=""
  env $envs timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline $bargs > $out/sweep_$i.json 2> $out/sweep_$i.err || { echo "failed: $cfg"; tail -5 $out/sweep_$i.err; exit 1; }
  python - $out/sweep_$i.json "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], "| value", d["value"], "| k1", k["k1_GBps"], "k1 ms", k["k1_ms_per_batch"], "| gates ms", k["gates_ms_per_batch"], "| k2 ms", k["k2_ms_per_batch"], "k2 GB/s", k["k2_GBps_on_item_bytes"], "| dev", k["k1_gates_k2_GBps"], "| h2d", d["pipeline"]["h2d_GBps"])
PY
done
