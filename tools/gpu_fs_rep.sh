#!/bin/bash
# configs[0] e2e fs, three repeats (separate processes) on one box.
set -o pipefail
out=gpurun_out/${1:-fsrep}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TSG_LAYER_PROF=1
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --e2e fs --steps 5 > $out/fs_$r.json 2> $out/fs_$r.err || { tail $out/fs_$r.err; exit 2; }
  python -c "import json; d=json.loads(open('$out/fs_$r.json').read().strip().splitlines()[-1]); print('fs', $r, d['value'], d['ms_per_step'], d['checks'])"
done
