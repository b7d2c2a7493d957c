#!/bin/bash
set -o pipefail
tools/gpu_tests.sh r2f && tools/gpu_sweep.sh r2sw3 "TSG_K2_DIAG=1|" "TSG_NONE=0|--batch-mib 2048" && \
TSG_K2_DIAG=1 timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2sw3/diag.json 2>&1
