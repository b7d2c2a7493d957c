#!/bin/bash
# K2 per-entry trace (tools/k2trace.py) of the builtin rules; with TSG_LIB_VARIANT=<a
# K2_TRACE_PHASE build> also the phases of each entry.  usage: tools/gpu_k2trace.sh TAG
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u tools/k2trace.py run $out/k2t 1024 > $out/k2t.log 2>&1 || { tail $out/k2t.log; exit 1; }
python tools/k2trace.py report $out/k2t --phases > $out/k2t_report.json || exit 2
python3 -c "
import json; d=json.load(open('$out/k2t_report.json'))
print({k: v for k, v in d.items() if k in ('span_us', 'dur_us', 'start_us', 'end_us', 'us_per_item', 'meta', 'phases_us_p50', 'phases_us_mean')})
"
