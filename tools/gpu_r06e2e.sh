#!/bin/bash
# Round 6: the GPU suite, then e2e layer / fs (three runs each) and one TSG_PROF layer run
# (resolution phases per piece).
set -o pipefail
out=gpurun_out/r06/${1:-e2e2}
mkdir -p $out
echo "== gpu suite" && timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2 3; do
  for k in layer fs; do
    timeout -k 10 300 python -u bench.py --e2e $k --steps 3 > $out/${k}_$i.json 2> $out/${k}_$i.err || { tail $out/${k}_$i.err; exit 2; }
    echo "$k run $i $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['unpipelined'])" $out/${k}_$i.json)"
  done
done
TSG_PROF=1 timeout -k 10 300 python -u bench.py --e2e layer --steps 2 --no-cpu-baseline > $out/prof_layer.json 2> $out/prof_layer.err || { tail $out/prof_layer.err; exit 3; }
grep "resolve: setup" $out/prof_layer.err | tail -8
echo done
