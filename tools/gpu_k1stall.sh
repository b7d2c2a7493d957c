#!/bin/bash
# K1 stall breakdown (one SQ pass: wave cycles, waits, active instruction cycles) on
# tools/kab.py's 1 GiB builtin batch.  usage: tools/gpu_k1stall.sh TAG
set -o pipefail
out=gpurun_out/${1:-k1stall}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES \
  --output-format csv -d $out/sq_stall -o run -- python tools/kab.py 1024 3 > $out/kab_stall.log 2>&1 || exit 3
tail -1 $out/kab_stall.log
