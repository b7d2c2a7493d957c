#!/bin/bash
# K2 change check: the GPU parity suite, kernel-only timings (builtin, user1000) and a K2
# entry trace of the builtin batch.  usage: tools/gpu_k2round.sh TAG
set -o pipefail
out=gpurun_out/${1:-k2r}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for r in builtin user1000; do
  timeout -k 10 200 python -u tools/kab.py 1024 7 --rules $r > $out/kab_$r.json 2> $out/kab_$r.err || { tail -5 $out/kab_$r.err; exit 2; }
  cat $out/kab_$r.json
done
timeout -k 10 300 python -u tools/k2trace.py run $out/k2b 1024 > $out/k2b.log 2>&1 || { tail $out/k2b.log; exit 3; }
python tools/k2trace.py report $out/k2b > $out/k2b_report.json && python -c "import json; d=json.load(open('$out/k2b_report.json')); print('span', d['span_us'], 'slowest', d['slowest'][:3])"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_user1000 -o run -- python tools/kab.py 1024 3 --rules user1000 > $out/prof_user1000.log 2>&1 || exit 4
f=$(find $out/prof_user1000 -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 $f | head -12
