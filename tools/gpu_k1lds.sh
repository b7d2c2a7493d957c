#!/bin/bash
# K1 LDS utilisation on the GPU box: one SQ pass with the LDS-array busy counter beside the
# instruction mix, on tools/kab.py's 1 GiB builtin batch.  usage: tools/gpu_k1lds.sh TAG
set -o pipefail
out=gpurun_out/${1:-k1lds}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d $out/sq -o run -- python tools/kab.py 1024 3 > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 3; }
tail -1 $out/sq.log
