#!/bin/bash
set -o pipefail
out=gpurun_out/r05/kv1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in default nover tileonly ldsonly loadonly; do
  if [ $v = default ]; then unset TSG_LIB_VARIANT; else export TSG_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/kab.py 1024 7 > $out/kab_$v.json 2> $out/kab_$v.err || { echo "fail $v"; tail $out/kab_$v.err; exit 1; }
  echo $v; cat $out/kab_$v.json
done
unset TSG_LIB_VARIANT
echo "== SQ" && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY --output-format csv -d $out/pmc_sq -o run -- \
  python tools/kab.py 1024 3 > $out/pmc_sq.out 2>&1 || { tail $out/pmc_sq.out; exit 2; }
python tools/sq_summary.py $out/pmc_sq/run_counter_collection.csv k1f --bytes 1073741824
echo "== SQ2" && timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_sq2 -o run -- \
  python tools/kab.py 1024 3 > $out/pmc_sq2.out 2>&1 || { tail $out/pmc_sq2.out; exit 3; }
python tools/sq_summary.py $out/pmc_sq2/run_counter_collection.csv k1f --bytes 1073741824
echo done
