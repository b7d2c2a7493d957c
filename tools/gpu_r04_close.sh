#!/bin/bash
# Round-4 closing evidence: GPU tests, smoke, configs[1] / configs[3] benches with kernel
# traces, FETCH_SIZE and SQ passes (profiles/pmc records), configs[4] bench.
set -o pipefail
out=gpurun_out/${1:-r04/close}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 2; }
tail -1 $out/smoke.log
bash tools/gpu_bench_prof.sh ${1:-r04/close}/bench || exit 3
bash tools/gpu_bench_prof.sh ${1:-r04/close}/u1000 --rules user1000 --cpu-mib 256 || exit 4
echo "== bench allow-exclude" && timeout -k 10 400 python -u bench.py --rules allow-exclude > $out/bench_allow.json 2> $out/bench_allow.err || { tail $out/bench_allow.err; exit 5; }
head -c 400 $out/bench_allow.json; echo
echo done
