#!/bin/bash
# K1F iteration: its parity tests, kernel-only timing (tools/kab.py), a short configs[1] bench
# line and a rocprofv3 kernel trace of it.  usage: tools/gpu_k1f_kab.sh TAG
set -o pipefail
tag=${1:-k1fk}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== k1f tests" && timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "k1_matches or k1f_ or adaptation or corpus_vs or slot_prefix" > $out/k1f_tests.log 2>&1 || { tail -40 $out/k1f_tests.log; exit 1; }
tail -1 $out/k1f_tests.log
echo "== kab" && timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab.json 2> $out/kab.err || { tail $out/kab.err; exit 2; }
cat $out/kab.json
echo "== bench" && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 3; }
python -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['roofline']['frac'], d['kernels']['k1_ms_per_batch'], d['kernels']['device_ms_per_batch'], d['roofline']['k1_gates_k2_frac'])"
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/trace.out 2>&1 || { tail $out/trace.out; exit 4; }
cut -c1-140 $out/trace/run_kernel_stats.csv | head -12
echo done
