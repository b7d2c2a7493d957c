#!/bin/bash
# SQ counters per kernel (one pass) over tools/kab.py, plus kab itself for the event count.
# usage: tools/gpu_sqitems.sh TAG
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 240 python -u tools/kab.py 1024 3 > $out/kab.json 2> $out/kab.err || { tail $out/kab.err; exit 1; }
cat $out/kab.json
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES \
  --output-format csv -d $out/sq -o run -- python tools/kab.py 1024 2 > $out/sq.log 2>&1 || { tail $out/sq.log; exit 2; }
python tools/sq_summary.py $out/sq/run_counter_collection.csv > $out/sq_summary.json || exit 3
cat $out/sq_summary.json | head -80

echo "== k2 trace"
timeout -k 10 300 python -u tools/k2trace.py run $out/k2t 1024 > $out/k2t.log 2>&1 || { tail $out/k2t.log; exit 4; }
python tools/k2trace.py report $out/k2t > $out/k2t_report.json || exit 5
head -c 3000 $out/k2t_report.json
echo "== k2 diag"
TSG_K2_DIAG=1 timeout -k 10 240 python -u tools/kab.py 1024 3 > $out/kab_diag.json 2> $out/kab_diag.err || { tail $out/kab_diag.err; exit 6; }
cat $out/kab_diag.json
echo done
