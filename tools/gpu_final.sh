#!/bin/bash
# Final check of HEAD: the GPU suite as the driver runs it, smoke, the default bench, and
# three e2e layer repeats.
set -o pipefail
out=gpurun_out/${1:-final}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 2; }
tail -1 $out/smoke.log
echo "== bench" && timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 3; }
python -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['kernels']['device_ms_per_batch'])"
export TSG_LAYER_PROF=1
for r in 1 2 3; do
  timeout -k 10 400 python -u bench.py --e2e layer --steps 3 > $out/layer_$r.json 2> $out/layer_$r.err || { tail $out/layer_$r.err; exit 4; }
  python -c "import json; d=json.loads(open('$out/layer_$r.json').read().strip().splitlines()[-1]); print('layer', $r, d['value'], d['ms_per_step'])"
done
