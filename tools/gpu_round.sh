#!/bin/bash
# Round evidence on one MI355X: GPU parity suite, smoke, headline bench + rocprofv3 kernel
# stats / FETCH_SIZE / SQ passes, configs[3] and configs[4] benches, configs[0] end to end.
# usage: tools/gpu_round.sh TAG     (every GPU step under its own limit; stops at a failure)
set -o pipefail
tag=${1:-r2}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "== tests" && timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -20 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
echo "== smoke" && timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 2; }
cat $out/smoke.log
tools/gpu_bench_prof.sh $tag || exit 3
# the headline line again, now with the FETCH_SIZE record of this device code (roofline.traffic)
mkdir -p profiles/pmc && cp $out/pmc_builtin.json profiles/pmc/builtin.json && \
  echo "== bench (with traffic)" && timeout -k 10 400 python -u bench.py > $out/bench_final.json 2> $out/bench_final.err || { tail $out/bench_final.err; exit 10; }
tail -c 1500 $out/bench_final.json
echo "== configs[3]" && timeout -k 10 400 python -u bench.py --rules user1000 --steps 2 --warmup 1 --cpu-mib 16 > $out/bench_user1000.json 2> $out/bench_user1000.err || { tail $out/bench_user1000.err; exit 4; }
echo "== configs[4]" && timeout -k 10 400 python -u bench.py --rules allow-exclude --steps 2 --warmup 1 --cpu-mib 256 > $out/bench_allow.json 2> $out/bench_allow.err || { tail $out/bench_allow.err; exit 5; }
echo "== configs[0]" && timeout -k 10 400 python -u tools/fs_bench.py > $out/fs_bench.json 2> $out/fs_bench.err || { tail $out/fs_bench.err; exit 6; }
echo "== configs[2] shape" && timeout -k 10 400 python -u tools/layer_bench.py 2 3 > $out/layer_bench.json 2> $out/layer_bench.err || { tail $out/layer_bench.err; exit 7; }
echo "== e2e fs" && timeout -k 10 300 python -u bench.py --e2e fs --steps 3 > $out/e2e_fs.json 2> $out/e2e_fs.err || { tail $out/e2e_fs.err; exit 8; }
echo "== e2e layer" && timeout -k 10 300 python -u bench.py --e2e layer --steps 3 > $out/e2e_layer.json 2> $out/e2e_layer.err || { tail $out/e2e_layer.err; exit 9; }
echo done
