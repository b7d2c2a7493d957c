#!/bin/bash
set -o pipefail
tools/gpu_tests.sh r2h && tools/gpu_sweep.sh r2sw5 "TSG_NONE=0|" "TSG_K1_GRID=4|" "TSG_K1_GRID=8|" "TSG_NONE=0|--batch-mib 2048"
