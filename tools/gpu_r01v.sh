set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for v in nolds coal coalnolds noruns nocls; do
TSG_LIB_VARIANT=$v timeout -k 10 300 python -u tools/k1sweep.py 4 0 >> gpurun_out/k1var.log 2>&1
done
TSG_K1_NS=8 timeout -k 10 300 python -u tools/k1sweep.py 4 ns8 >> gpurun_out/k1var.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/prof/ps -o ps --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/ps.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d gpurun_out/prof/ps2 -o ps2 --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/ps2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pf -o pf --output-format csv -- python3 tools/kprof.py 4 1 > gpurun_out/prof/pf.log 2>&1
