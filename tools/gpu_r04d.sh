#!/bin/bash
# Round 4: GPU tests, the headline bench (device time per batch), e2e fs (configs[0]),
# e2e fs at configs[4]'s mix, e2e layer (configs[2] shape).
set -o pipefail
out=gpurun_out/${1:-r04d}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== bench" && timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 2; }
python -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); k=d['kernels']
print(d['value'], {x:k[x] for x in k if 'ms' in x and 'per_batch' in x})"
export TSG_LAYER_PROF=1
echo "== e2e fs" && timeout -k 10 300 python -u bench.py --e2e fs --steps 3 > $out/e2e_fs.json 2> $out/e2e_fs.err || { tail $out/e2e_fs.err; exit 3; }
head -c 600 $out/e2e_fs.json; echo; grep -E "^(fs|pieces|layer)" $out/e2e_fs.err | tail -4
echo "== e2e fs configs[4] mix" && timeout -k 10 300 python -u bench.py --e2e fs --steps 3 --rules allow-exclude --binary-frac 0.3 --binary-text-head 0.5 > $out/e2e_fs_c4.json 2> $out/e2e_fs_c4.err || { tail $out/e2e_fs_c4.err; exit 4; }
head -c 600 $out/e2e_fs_c4.json; echo
echo "== e2e layer" && timeout -k 10 400 python -u bench.py --e2e layer --steps 3 > $out/e2e_layer.json 2> $out/e2e_layer.err || { tail $out/e2e_layer.err; exit 5; }
head -c 600 $out/e2e_layer.json; echo
echo done
