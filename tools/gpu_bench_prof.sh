#!/bin/bash
# Bench + rocprofv3 evidence on the GPU box.  usage: tools/gpu_bench_prof.sh TAG [bench args]
# Every GPU step runs under its own time limit; the script stops at the first failure.
# TAG is a path under gpurun_out/ and profiles/ (e.g. r03/b1); the FETCH_SIZE pass is recorded
# in $out/pmc_<rules>.json for profiles/pmc/ (bench.py's roofline.traffic).
set -o pipefail
tag=${1:-r2}; shift
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== bench" && timeout -k 10 400 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err || exit 1
tail -c 3000 $out/bench.json
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $out/trace.out 2>&1 || exit 2
echo "== FETCH_SIZE" && timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $out/pmc_fetch.out 2>&1 || exit 3
echo "== SQ" && timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY --output-format csv -d $out/pmc_sq -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $out/pmc_sq.out 2>&1 || exit 4
rules=builtin
for a in "$@"; do case "$prev" in --rules) rules=$a;; esac; prev=$a; done
python tools/pmc_traffic.py --record $rules $out/pmc_fetch/run_counter_collection.csv $out/bench.json \
  profiles/$tag/bench_pmc_fetch.csv > $out/pmc_$rules.json || exit 5
cat $out/pmc_$rules.json
echo done
