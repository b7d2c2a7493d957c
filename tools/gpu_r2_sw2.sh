#!/bin/bash
set -o pipefail
tools/gpu_tests.sh r2e && tools/gpu_sweep.sh r2sw2 "TSG_NONE=0|" "TSG_K1_GRID=4|" "TSG_NONE=0|--batch-mib 2048" && \
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib -o calib -- tools/fetch_calib > gpurun_out/calib.out 2>&1
