#!/bin/bash
# e2e ingest + scan benches with stage profiles (TSG_LAYER_PROF).  usage: tools/gpu_e2e.sh TAG
set -o pipefail
tag=${1:-e2e}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TSG_LAYER_PROF=1
echo "== e2e fs" && timeout -k 10 300 python -u bench.py --e2e fs --steps 3 > $out/e2e_fs.json 2> $out/e2e_fs.err || { tail $out/e2e_fs.err; exit 2; }
cat $out/e2e_fs.json; grep -E "^(fs|pieces|layer)" $out/e2e_fs.err | tail -4
echo "== e2e layer" && timeout -k 10 400 python -u bench.py --e2e layer --steps 3 > $out/e2e_layer.json 2> $out/e2e_layer.err || { tail $out/e2e_layer.err; exit 3; }
cat $out/e2e_layer.json; grep -E "^(fs|pieces|layer)" $out/e2e_layer.err | tail -4
echo done
