#!/bin/bash
set -o pipefail
tools/gpu_tests.sh r2g && tools/gpu_sweep.sh r2sw4 "TSG_K2_DIAG=1|" "TSG_NONE=0|--batch-mib 2048" "TSG_NONE=0|--batch-mib 5120"
