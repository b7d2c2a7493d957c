#!/bin/bash
# e2e fs (configs[0]) per piece floor (tsg_test_knob piece_mib).  usage: tools/gpu_fs_pieces.sh TAG MiB...
set -o pipefail
out=gpurun_out/${1:-fsp}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TSG_LAYER_PROF=1
for m in "$@"; do
  echo "== piece $m" && timeout -k 10 300 python -u bench.py --e2e fs --steps 5 --piece-mib $m > $out/fs_$m.json 2> $out/fs_$m.err || { tail $out/fs_$m.err; exit 2; }
  python -c "import json; d=json.loads(open('$out/fs_$m.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
  grep -E "^(fs|pieces|fs_scan)" $out/fs_$m.err | tail -3
done
