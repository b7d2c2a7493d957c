#!/bin/bash
# Round-4 evidence: configs[1] (builtin) and configs[3] (user1000, 256 MiB CPU sample) benches
# with kernel traces, FETCH_SIZE and SQ passes (tools/gpu_bench_prof.sh).
set -o pipefail
bash tools/gpu_bench_prof.sh r04/bench || exit $?
bash tools/gpu_bench_prof.sh r04/u1000 --rules user1000 --cpu-mib 256 || exit $?
