#!/bin/bash
# e2e fs (configs[0]), fs at configs[4]'s mix, layer (configs[2] shape), each twice.
set -o pipefail
out=gpurun_out/${1:-e2e4}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TSG_LAYER_PROF=1
for r in 1 2; do
echo "== e2e fs $r" && timeout -k 10 300 python -u bench.py --e2e fs --steps 5 > $out/e2e_fs_$r.json 2> $out/e2e_fs_$r.err || { tail $out/e2e_fs_$r.err; exit 3; }
python -c "import json; d=json.loads(open('$out/e2e_fs_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
grep -E "^(pieces|fs_scan)" $out/e2e_fs_$r.err | tail -2
echo "== e2e fs configs[4] mix $r" && timeout -k 10 300 python -u bench.py --e2e fs --steps 5 --rules allow-exclude --binary-frac 0.3 --binary-text-head 0.5 > $out/e2e_fs_c4_$r.json 2> $out/e2e_fs_c4_$r.err || { tail $out/e2e_fs_c4_$r.err; exit 4; }
python -c "import json; d=json.loads(open('$out/e2e_fs_c4_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
grep -E "^(pieces|fs_scan)" $out/e2e_fs_c4_$r.err | tail -2
echo "== e2e layer $r" && timeout -k 10 400 python -u bench.py --e2e layer --steps 3 > $out/e2e_layer_$r.json 2> $out/e2e_layer_$r.err || { tail $out/e2e_layer_$r.err; exit 5; }
python -c "import json; d=json.loads(open('$out/e2e_layer_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
grep -E "^(pieces|layer_scan)" $out/e2e_layer_$r.err | tail -2
done
echo done
